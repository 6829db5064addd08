// h2s_preview.hip — the preview tail of the chain (src/utils.py:46-49,
// :719-765; src/preview.py:108-117): aspect-fit resize of the 8-bit yuv420p
// the chain produced, Y'CbCr -> RGB24 and the GUI's display gamma.
//
// The preview is latency-bound (a 4K frame is ~25 MB of RGB out), so these
// kernels are plain one-thread-per-output-sample gathers; blockIdx.z is the
// frame of a batch (extract_frames_with_conversion_batch, src/utils.py:668-716:
// N frames, one call); the tone-map work before them runs through k_tile.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "h2s_device.h"

namespace h2s {

// separable resize of one u8 plane, taps/weights precomputed on the host per
// output column (wx: ow x T, start sx) and row (wy: oh x T, start sy); source
// indices clamp at the edges (swscale's edge handling)
__global__ void k_resize_u8(const uint8_t* __restrict__ src, int sw, int sh, long long sls, long long sfp,
                            uint8_t* __restrict__ dst, int ow, int oh, long long dls, long long dfp,
                            const float* __restrict__ wx, const int* __restrict__ sx,
                            const float* __restrict__ wy, const int* __restrict__ sy, int T) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= ow || y >= oh) return;
  src += blockIdx.z * sfp;
  dst += blockIdx.z * dfp;
  float acc = 0.0f;
  for (int j = 0; j < T; j++) {
    int r = sy[y] + j;
    r = r < 0 ? 0 : (r > sh - 1 ? sh - 1 : r);
    const uint8_t* row = src + r * sls;
    float h = 0.0f;
    for (int i = 0; i < T; i++) {
      int c = sx[x] + i;
      c = c < 0 ? 0 : (c > sw - 1 ? sw - 1 : c);
      h = fmaf(wx[x * T + i], (float)row[c], h);
    }
    acc = fmaf(wy[y * T + j], h, acc);
  }
  const float v = floorf(acc + 0.5f);
  dst[y * dls + x] = (uint8_t)(v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v));
}

// yuv420p (BT.709, limited) -> RGB24 full range, chroma of pixel (x, y) from
// sample (x/2, y/2); then the display-gamma LUT
__global__ void k_yuv8_rgb24(const uint8_t* __restrict__ yp, long long yls, const uint8_t* __restrict__ up,
                             const uint8_t* __restrict__ vp, long long cls, long long yuv_fp, int w, int h,
                             uint8_t* __restrict__ rgb, long long rls, long long rgb_fp,
                             const uint8_t* __restrict__ glut) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  yp += blockIdx.z * yuv_fp, up += blockIdx.z * yuv_fp, vp += blockIdx.z * yuv_fp;
  rgb += blockIdx.z * rgb_fp;
  const float Y = 1.16438356f * ((float)yp[y * yls + x] - 16.0f);
  const float U = (float)up[(y >> 1) * cls + (x >> 1)] - 128.0f;
  const float V = (float)vp[(y >> 1) * cls + (x >> 1)] - 128.0f;
  const float c[3] = {fmaf(1.79274107f, V, Y), fmaf(-0.53290933f, V, fmaf(-0.21324861f, U, Y)), fmaf(2.11240179f, U, Y)};
  uint8_t* o = rgb + y * rls + 3 * x;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float v = floorf(c[k] + 0.5f);
    o[k] = glut[(int)(v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v))];
  }
}

hipError_t launch_resize_u8(const uint8_t* src, int sw, int sh, long long sls, long long sfp, uint8_t* dst, int ow,
                            int oh, long long dls, long long dfp, const float* wx, const int* sx, const float* wy,
                            const int* sy, int T, int nframes, hipStream_t s) {
  hipLaunchKernelGGL(k_resize_u8, dim3((ow + 255) / 256, oh, nframes), dim3(256), 0, s, src, sw, sh, sls, sfp, dst, ow,
                     oh, dls, dfp, wx, sx, wy, sy, T);
  return hipGetLastError();
}

hipError_t launch_yuv8_rgb24(const uint8_t* yp, long long yls, const uint8_t* up, const uint8_t* vp, long long cls,
                             long long yuv_fp, int w, int h, uint8_t* rgb, long long rls, long long rgb_fp,
                             const uint8_t* glut, int nframes, hipStream_t s) {
  hipLaunchKernelGGL(k_yuv8_rgb24, dim3((w + 255) / 256, h, nframes), dim3(256), 0, s, yp, yls, up, vp, cls, yuv_fp, w,
                     h, rgb, rls, rgb_fp, glut);
  return hipGetLastError();
}

}  // namespace h2s
