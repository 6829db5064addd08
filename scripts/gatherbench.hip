// gatherbench.hip — cost of one wave-wide gather instruction on gfx950 by
// lane->address pattern and load width (CU clocks per wave-instruction at
// the nominal 2.4 GHz; lower is better).  Table = 65^3 x 16 B (4.4 MB).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
#define ITERS 256
template <int W>  // W = bytes per lane: 4, 8, 12, 16
__global__ __launch_bounds__(256) void k_g(const float4* tab, int nbytes, const int* pat, float* out, int zero) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, nbytes, 0x00020000);
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
  int off[8];
  for (int k = 0; k < 8; k++) off[k] = pat[((wave * 8 + k) & 1023) * 64 + lane];
  float acc = 0.f;
  for (int i = 0; i < ITERS; i++) {
    const int t = ((i & 1) << 4) ^ ((i * zero) & 0x7ff0);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int o = off[k] ^ t;
      if (W == 16) { float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0)); acc += v.x + v.w; }
      else if (W == 12) { typedef float v3 __attribute__((ext_vector_type(3))); v3 v = __builtin_amdgcn_raw_buffer_load_b96(r, o, 0, 0); acc += v.x + v.z; }
      else if (W == 8) { typedef float v2 __attribute__((ext_vector_type(2))); v2 v = __builtin_bit_cast(v2, __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 0)); acc += v.x + v.y; }
      else { acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0)); }
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
  const char* names[] = {"same addr", "coalesced 16B", "1 lane/64B", "1 lane/128B", "stride 1040B",
                         "random 4.4MB", "random 32KB", "random 1MB", "4 lanes/rec rand", "smooth-like"};
  srand(1);
  for (int p = 0; p < 10; p++) {
    for (int w = 0; w < 1024; w++) {
      int base = (rand() % (n - 4096)) & ~63;
      int grp = rand() % (n - 64);
      for (int l = 0; l < 64; l++) {
        int rec;
        switch (p) {
          case 0: rec = base; break;
          case 1: rec = base + l; break;
          case 2: rec = base + 4 * l; break;
          case 3: rec = (base + 8 * l) % n; break;
          case 4: rec = (base + 65 * l) % n; break;
          case 5: rec = rand() % n; break;
          case 6: rec = rand() % 2048; break;
          case 7: rec = rand() % 65536; break;
          case 8: rec = (l % 4 == 0) ? rand() % n : -1; break;
          default: { int t = grp + (l / 4) * 1 + ((l & 3) >> 1) * 65 + (l & 1) * 4225; rec = t % n; }
        }
        if (rec < 0) rec = h[w * 64 + l - 1] / 16;
        h[w * 64 + l] = (rec & ~1) * 16;
      }
    }
    CHK(hipMemcpy(pat, h, 1024 * 64 * 4, hipMemcpyHostToDevice));
    for (int wi = 0; wi < 4; wi++) {
      hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
      float best = 1e30f;
      for (int r = 0; r < 4; r++) {
        CHK(hipEventRecord(a));
        if (wi == 0) hipLaunchKernelGGL(k_g<16>, dim3(blocks), dim3(256), 0, 0, tab, nbytes, pat, out, 0);
        if (wi == 1) hipLaunchKernelGGL(k_g<12>, dim3(blocks), dim3(256), 0, 0, tab, nbytes, pat, out, 0);
        if (wi == 2) hipLaunchKernelGGL(k_g<8>, dim3(blocks), dim3(256), 0, 0, tab, nbytes, pat, out, 0);
        if (wi == 3) hipLaunchKernelGGL(k_g<4>, dim3(blocks), dim3(256), 0, 0, tab, nbytes, pat, out, 0);
        CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
        float ms; CHK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
      }
      double instr = (double)blocks * 4 * ITERS * 8;
      double clk_per = best * 1e-3 * 2.4e9 * 256 / instr;
      printf("%-18s x%-2d  %8.3f ms  %7.2f clk/wave-instr/CU\n", names[p], wi == 0 ? 16 : wi == 1 ? 12 : wi == 2 ? 8 : 4, best, clk_per);
    }
  }
  return 0;
}
