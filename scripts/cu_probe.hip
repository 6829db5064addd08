// Which compute unit runs which block: k_tile-shaped blocks (256 threads,
// 27.6 KB LDS) record their XCC / SE / SH / CU ids and their start time,
// spinning long enough that every resident block overlaps.
// Usage: cu_probe NBLOCKS > out.txt   (one line per block: b xcc se sh cu t0)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void k_probe(unsigned* out, unsigned long long* t, int spin) {
  extern __shared__ float lds[];
  lds[threadIdx.x] = 0.0f;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20); // HW_REG_XCC_ID
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    t[blockIdx.x] = t0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(10);
  }
  __syncthreads();
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 1280;
  const int spin = argc > 2 ? atoi(argv[2]) : 20000;   // 100 MHz ticks: 200 us
  unsigned* d;
  unsigned long long* dt;
  hipMalloc(&d, 8 * nb);
  hipMalloc(&dt, 8 * nb);
  hipLaunchKernelGGL(k_probe, dim3(nb), dim3(256), 28260, 0, d, dt, spin);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<unsigned> h(2 * nb);
  std::vector<unsigned long long> ht(nb);
  hipMemcpy(h.data(), d, 8 * nb, hipMemcpyDeviceToHost);
  hipMemcpy(ht.data(), dt, 8 * nb, hipMemcpyDeviceToHost);
  unsigned long long tmin = ~0ull;
  for (auto v : ht) tmin = v < tmin ? v : tmin;
  for (int b = 0; b < nb; b++) {
    const unsigned hw = h[2 * b];
    printf("%d %u %u %u %u %llu\n", b, h[2 * b + 1] & 15, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15, ht[b] - tmin);
  }
  return 0;
}
