// gathermask.hip — does an exec-masked wave gather cost less than a full
// one on gfx950?  CU clocks per wave-instruction (at 2.4 GHz nominal) of a
// 12-byte buffer gather with k of 64 lanes active (the others skip the load
// under exec), on the "same address" and the "smooth-like" lane->record
// patterns of gatherbench.hip.  Table = 65^3 x 16 B.  (Prices the
// round-4 lattice-dedup ideas: a step that serves most lanes from scalar or
// quad-shared records only pays if a masked gather is cheaper.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
#define ITERS 256
typedef float v3 __attribute__((ext_vector_type(3)));
__global__ __launch_bounds__(256) void k_g(const float4* tab, int nbytes, const int* pat, float* out, int zero,
                                           unsigned long long mask) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, nbytes, 0x00020000);
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
  const bool on = (mask >> lane) & 1ull;
  int off[8];
  for (int k = 0; k < 8; k++) off[k] = pat[((wave * 8 + k) & 1023) * 64 + lane];
  float acc = 0.f;
  for (int i = 0; i < ITERS; i++) {
    const int t = ((i & 1) << 4) ^ ((i * zero) & 0x7ff0);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int o = off[k] ^ t;
      if (on) {
        v3 v = __builtin_amdgcn_raw_buffer_load_b96(r, o, 0, 0);
        acc += v.x + v.z;
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
int main() {
  const int n = 65 * 65 * 65, nbytes = n * 16, blocks = 2048;
  float4* tab; int* pat; float* out;
  CHK(hipMalloc(&tab, nbytes)); CHK(hipMemset(tab, 0, nbytes));
  CHK(hipMalloc(&out, blocks * 256 * 4));
  CHK(hipMalloc(&pat, 1024 * 64 * 4));
  int* h = (int*)malloc(1024 * 64 * 4);
  const char* names[] = {"same addr", "smooth-like", "random 4.4MB"};
  const unsigned long long masks[] = {~0ull, 0x00000000FFFFFFFFull, 0x000000000000FFFFull, 0x1111111111111111ull,
                                      0x0101010101010101ull, 0x0000000000000001ull, 0x5555555555555555ull};
  const char* mnames[] = {"64 lanes", "32 (lo half)", "16 (first row)", "16 (1 per quad)", "8 (1 per 8)", "1 lane",
                          "32 (every 2nd)"};
  srand(1);
  for (int p = 0; p < 3; p++) {
    for (int w = 0; w < 1024; w++) {
      int base = (rand() % (n - 4096)) & ~63;
      int grp = rand() % (n - 64);
      for (int l = 0; l < 64; l++) {
        int rec;
        if (p == 0) rec = base;
        else if (p == 1) { int t = grp + (l / 4) * 1 + ((l & 3) >> 1) * 65 + (l & 1) * 4225; rec = t % n; }
        else rec = rand() % n;
        h[w * 64 + l] = (rec & ~1) * 16;
      }
    }
    CHK(hipMemcpy(pat, h, 1024 * 64 * 4, hipMemcpyHostToDevice));
    for (int m = 0; m < 7; m++) {
      hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
      float best = 1e30f;
      for (int rep = 0; rep < 4; rep++) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(k_g, dim3(blocks), dim3(256), 0, 0, tab, nbytes, pat, out, 0, masks[m]);
        CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
        float ms; CHK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
      }
      double instr = (double)blocks * 4 * ITERS * 8;
      printf("%-14s %-16s %8.3f ms  %7.2f clk/wave-instr/CU\n", names[p], mnames[m], best, best * 1e-3 * 2.4e9 * 256 / instr);
    }
  }
  return 0;
}
