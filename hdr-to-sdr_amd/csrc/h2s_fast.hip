// h2s_fast.hip — launcher of the tile kernel (h2s_tile.h): the product
// instances, the dispatch over every instance, and the Y'CbCr lattice build.
#include <hip/hip_runtime.h>

#include "h2s_tile.h"

namespace h2s {

H2S_TILE_INSTANCE(0, 0)
H2S_TILE_EXTERN(0, 1)   // h2s_fast_lp.hip
H2S_TILE_EXTERN(1, 0)
H2S_TILE_EXTERN(1, 1)
H2S_TILE_EXTERN(2, 0)
H2S_TILE_EXTERN(2, 1)
H2S_TILE_EXTERN(3, 0)
H2S_TILE_EXTERN(3, 1)
H2S_TILE_EXTERN(4, 0)
H2S_TILE_EXTERN(4, 1)
H2S_TILE_EXTERN(5, 0)
H2S_TILE_EXTERN(5, 1)

// YUV-premultiplied lattice (12-byte records, .cube order):
// ((16 + 219*Y)*s + 0.5, 224*s*Cb/4, 224*s*Cr/4) with Y, Cb, Cr the BT.709
// values of the clamped RGB lattice point, in the oracle's S6 operation order.
__global__ void k_build_lut_yuv(const float4* rgb, float* yuv, int n3, const YuvLutConsts K) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n3) return;
  const float4 c = rgb[i];
  const float R = clamp01(c.x), G = clamp01(c.y), B = clamp01(c.z);
  const float Y = K.k709[0] * R + K.k709[1] * G + K.k709[2] * B;
  const float cb = K.kcb[0] * R + K.kcb[1] * G + K.kcb[2] * B;
  const float cr = K.kcr[0] * R + K.kcr[1] * G + K.kcr[2] * B;
  const float s = K.s;
  if (K.rgb) {  // plain R'G'B' (libplacebo branch): lut3d's own lattice values, unclamped
    yuv[3 * i] = c.x, yuv[3 * i + 1] = c.y, yuv[3 * i + 2] = c.z;
    return;
  }
  // (H2S_EQMAGIC: no +0.5, k_tile rounds to nearest instead)
  yuv[3 * i] = (16.0f + 219.0f * Y) * s + (H2S_EQMAGIC ? 0.0f : 0.5f);
  yuv[3 * i + 1] = 224.0f * s * 0.25f * cb;
  yuv[3 * i + 2] = 224.0f * s * 0.25f * cr;
}

bool fast_supported(int tonemap) { return tonemap >= 4 && tonemap <= 8; }

// desat: 0 off, 1 weighted luma, 2 RGB-coefficient luma (vf_tonemap's; the
// libplacebo curves have none).  lp: the libplacebo branch (every operator).
// dbg: 0 = the
// product kernel; 1..5 = its debug instance for that h2s_stage (F.dbg set)
hipError_t launch_fast(const FastParams& F, int trc, int tm, int desat, int lp, hipStream_t s, int dbg) {
  const long long nt = (long long)F.nbx * F.nby * F.nframes;
  if (nt == 0) return hipSuccess;
  const long long nb = (nt + F.tpb - 1) / F.tpb;
  dim3 grid((unsigned)nb);
  // (5 blocks per CU, the LDS bound; 4 and 3, forced by padding this
  // allocation, measured +4 % and +42 % on the bench content:
  // profiles/r03/ablations/blocks_per_cu.log)
  const size_t lds = ((size_t)F.eq_n * sizeof(uint16_t) + 15) & ~(size_t)15;
  if (tm == 7 || tm == 8 || lp) desat = 0;
#define H2S_DISPATCH(D) \
  return lp ? launch_tile<D, 1>(F, trc, tm, desat, grid, lds, s) : launch_tile<D, 0>(F, trc, tm, desat, grid, lds, s)
  switch (dbg) {
    case 0: H2S_DISPATCH(0);
    case 1: H2S_DISPATCH(1);
    case 2: H2S_DISPATCH(2);
    case 3: H2S_DISPATCH(3);
    case 4: H2S_DISPATCH(4);
    default: H2S_DISPATCH(5);
  }
#undef H2S_DISPATCH
}

hipError_t build_lut_yuv(const float4* rgb, float* yuv, int n, const YuvLutConsts& K, hipStream_t st) {
  const int n3 = n * n * n;
  hipLaunchKernelGGL(k_build_lut_yuv, dim3((n3 + 255) / 256), dim3(256), 0, st, rgb, yuv, n3, K);
  return hipGetLastError();
}

}  // namespace h2s
