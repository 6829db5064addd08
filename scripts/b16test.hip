// Does v_lshlrev_b16 (VOP2, gfx950) zero or preserve the destination's upper 16 bits?
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  unsigned v = 0x4B40ABCDu + threadIdx.x, d = 0xDEAD0000u;
  asm volatile("v_lshlrev_b16 %0, 4, %1" : "+v"(d) : "v"(v));
  out[threadIdx.x] = d;
}
int main() {
  unsigned* o;
  hipMalloc(&o, 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
  unsigned h[64];
  hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
  printf("in 0x%08x -> 0x%08x (%s)\n", 0x4B40ABCDu, h[0],
         (h[0] >> 16) == 0 ? "upper zeroed" : ((h[0] >> 16) == 0xDEAD ? "upper preserved" : "upper = source"));
  return 0;
}
