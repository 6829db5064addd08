// h2s_kernels.hip — gfx950 kernels for the HDR->SDR hot path.
//
// k_process: the whole per-frame chain of src/utils.py:38-42 fused into one
// pass over HBM: read packed 10/12-bit planar 4:2:0, upsample chroma, S1..S4
// per pixel, RGB->Y'CbCr, 2x2 chroma reduction, quantise, eq, write 4:2:0.
// One work item = QPT horizontally adjacent 2x2 luma quads (one output chroma
// sample each) of one chroma row of one frame; the flattened item index runs
// columns fastest, so a wavefront reads contiguous row segments (16-B Y loads,
// 8-B chroma loads per lane).  Blocks are remapped so that each XCD walks a
// contiguous range of rows (chroma halo rows and LUT lines stay in its L2).
#include <hip/hip_runtime.h>

#include <vector>

#include "h2s_device.h"
#include "h2s_lpx.h"
#include "h2s_peak.h"

namespace h2s {

// the upsampler's edge rule (params.chroma_edge; oracle/h2s_oracle.c edge())
__device__ __forceinline__ int edge(const KParams& P, int i, int n) { return chroma_edge_at(i, n, P.chroma_edge); }

// XCD-aware block remap: hardware deals blocks round-robin over 8 XCDs;
// give XCD x the contiguous logical range [x*per(+rem), ...).  Bijective.
__device__ __forceinline__ long long xcd_remap(long long b, long long nb) {
  const long long xcd = b & 7, idx = b >> 3, per = nb >> 3, rem = nb & 7;
  return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

__device__ __forceinline__ int ld16(const uint8_t* row, int x) {
  return *reinterpret_cast<const uint16_t*>(row + 2 * x);
}

// C444: BICUBIC chroma (two-pass path): store every pixel's (Cb, Cr) into
// P.chr444 (frame 0 of the launch, W x H) instead of the 2x2 mean; the
// chroma planes are then written by k_chroma_bicubic
// LPX: the libplacebo branch, stages 1-3 in exact arithmetic (h2s_lpx.h)
// from the integer codes (cc*: the chroma codes kept for it)
template <int QPT, bool VEC, bool OUT8, bool C444 = false, bool DYN = false, bool LPX = false>
__global__ __launch_bounds__(256) void k_process(const KParams P0) {
  LpX X;
  auto body = [&](const KParams& P, const int f, const int cy, const int cx0) {
  const int cw = P.cw, ch = P.ch;

  // ---- chroma: rows cy-1, cy, cy+1; columns cx0 .. cx0+QPT (halo) ----
  float cu[3][QPT + 1], cv[3][QPT + 1];
  int ccu[3][QPT + 1], ccv[3][QPT + 1];
  const int crow[3] = {edge(P, cy - 1, ch), cy, edge(P, cy + 1, ch)};
  const bool full = cx0 + QPT <= cw;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const uint8_t* ru = P.in[1] + f * P.in_fp[1] + crow[i] * P.in_ls[1];
    const uint8_t* rv = P.in[2] + f * P.in_fp[2] + crow[i] * P.in_ls[2];
    if (VEC && full && QPT == 4) {
      const uint2 a = *reinterpret_cast<const uint2*>(ru + 2 * cx0);
      const uint2 b = *reinterpret_cast<const uint2*>(rv + 2 * cx0);
      const int hx = edge(P, cx0 + 4, cw);
      const int m = (int)P.in_mask;   // h2s_lp_p010 TRUNCATE drops the two low bits
      int su[5] = {(int)(a.x & 0xffff) & m, (int)(a.x >> 16) & m, (int)(a.y & 0xffff) & m, (int)(a.y >> 16) & m,
                   ld16(ru, hx) & m};
      int sv[5] = {(int)(b.x & 0xffff) & m, (int)(b.x >> 16) & m, (int)(b.y & 0xffff) & m, (int)(b.y >> 16) & m,
                   ld16(rv, hx) & m};
#pragma unroll
      for (int k = 0; k <= QPT; k++) ccu[i][k] = su[k], ccv[i][k] = sv[k];
    } else {
#pragma unroll
      for (int k = 0; k <= QPT; k++) {
        const int x = edge(P, cx0 + k, cw);
        ccu[i][k] = ld16(ru, x) & (int)P.in_mask;
        ccv[i][k] = ld16(rv, x) & (int)P.in_mask;
      }
    }
#pragma unroll
    for (int k = 0; k <= QPT; k++) {
      cu[i][k] = (float)ccu[i][k] * P.c_scale + P.c_off;
      cv[i][k] = (float)ccv[i][k] * P.c_scale + P.c_off;
    }
  }
  // horizontal pass (left siting): h[2k] = c[k], h[2k+1] = (c[k] + c[k+1]) / 2
  float hu[3][2 * QPT], hv[3][2 * QPT];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int k = 0; k < QPT; k++) {
      hu[i][2 * k] = cu[i][k];
      hu[i][2 * k + 1] = 0.5f * cu[i][k] + 0.5f * cu[i][k + 1];
      hv[i][2 * k] = cv[i][k];
      hv[i][2 * k + 1] = 0.5f * cv[i][k] + 0.5f * cv[i][k + 1];
    }

  // ---- luma: rows 2cy, 2cy+1; columns 2cx0 .. 2cx0+2QPT-1 ----
  const int x0 = 2 * cx0;
  int ys[2][2 * QPT];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint8_t* ry = P.in[0] + f * P.in_fp[0] + (2 * cy + j) * P.in_ls[0];
    if (VEC && full && QPT == 4) {
      const uint4 a = *reinterpret_cast<const uint4*>(ry + 2 * x0);
      const unsigned w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        ys[j][2 * k] = (int)(w[k] & 0xffff & P.in_mask);
        ys[j][2 * k + 1] = (int)((w[k] >> 16) & P.in_mask);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2 * QPT; k++) {
        const int x = x0 + k < P.W ? x0 + k : P.W - 1;
        ys[j][k] = ld16(ry, x) & (int)P.in_mask;
      }
    }
  }

  // ---- per pixel chain, Y'CbCr, quantise ----
  int yo[2][2 * QPT], uo[QPT], vo[QPT];
#pragma unroll
  for (int k = 0; k < QPT; k++) {
    float cbs[4], crs[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
      const int j = p >> 1, x = 2 * k + (p & 1);
      const float cb = j == 0 ? 0.25f * hu[0][x] + 0.75f * hu[1][x] : 0.75f * hu[1][x] + 0.25f * hu[2][x];
      const float cr = j == 0 ? 0.25f * hv[0][x] + 0.75f * hv[1][x] : 0.75f * hv[1][x] + 0.25f * hv[2][x];
      const float yv = (float)ys[j][x] * P.y_scale + P.y_off;
      float r, g, b;
      const int px = 2 * (cx0 + k) + (p & 1), py = 2 * cy + j;
      if (LPX) {
        // the oracle's upsample_d: horizontal (left siting) then vertical, in double
        auto hx = [&](const int (&c)[3][QPT + 1], int i) -> double {
          const double a = lpx_chroma(P, c[i][x >> 1]);
          return (x & 1) ? 0.5 * (a + lpx_chroma(P, c[i][(x >> 1) + 1])) : a;
        };
        const double cbd = j == 0 ? 0.25 * hx(ccu, 0) + 0.75 * hx(ccu, 1) : 0.75 * hx(ccu, 1) + 0.25 * hx(ccu, 2);
        const double crd = j == 0 ? 0.25 * hx(ccv, 0) + 0.75 * hx(ccv, 1) : 0.75 * hx(ccv, 1) + 0.25 * hx(ccv, 2);
        lpx_chain<4>(P, X, lpx_luma(P, ys[j][x]), cbd, crd, px, py, r, g, b);
      } else {
        chain_px<4>(P, yv, cb, cr, r, g, b, lp_qoff(P, px, py));
      }
      r = clamp01(r), g = clamp01(g), b = clamp01(b);
      const float Y = P.k709[0] * r + P.k709[1] * g + P.k709[2] * b;
      cbs[p] = P.kcb[0] * r + P.kcb[1] * g + P.kcb[2] * b;
      crs[p] = P.kcr[0] * r + P.kcr[1] * g + P.kcr[2] * b;
      int yq = quant_o((16.0f + 219.0f * Y) * P.qscale, P.dither ? dither_off(px, py) : 0.5f, P.qmax);
      if (!P.eq_identity) yq = P.eq_lut[yq];
      yo[j][x] = expand_code(P, yq);
      if (C444 && px < P.W) P.chr444[(long long)py * P.W + px] = make_float2(cbs[p], crs[p]);
    }
    if (C444) continue;
    const float cb = ((cbs[0] + cbs[1]) + (cbs[2] + cbs[3])) * 0.25f;
    const float cr = ((crs[0] + crs[1]) + (crs[2] + crs[3])) * 0.25f;
    const float co = P.dither ? dither_off(cx0 + k, cy) : 0.5f;
    uo[k] = expand_code(P, quant_o((128.0f + 224.0f * cb) * P.qscale, co, P.qmax));
    vo[k] = expand_code(P, quant_o((128.0f + 224.0f * cr) * P.qscale, co, P.qmax));
  }

  // ---- stores ----
#pragma unroll
  for (int j = 0; j < 2; j++) {
    uint8_t* ry = P.out[0] + f * P.out_fp[0] + (2 * cy + j) * P.out_ls[0];
    if (VEC && full && QPT == 4) {
      if (OUT8) {
        uint2 w;
        w.x = (unsigned)yo[j][0] | ((unsigned)yo[j][1] << 8) | ((unsigned)yo[j][2] << 16) | ((unsigned)yo[j][3] << 24);
        w.y = (unsigned)yo[j][4] | ((unsigned)yo[j][5] << 8) | ((unsigned)yo[j][6] << 16) | ((unsigned)yo[j][7] << 24);
        *reinterpret_cast<uint2*>(ry + x0) = w;
      } else {
        uint4 w;
        w.x = (unsigned)yo[j][0] | ((unsigned)yo[j][1] << 16);
        w.y = (unsigned)yo[j][2] | ((unsigned)yo[j][3] << 16);
        w.z = (unsigned)yo[j][4] | ((unsigned)yo[j][5] << 16);
        w.w = (unsigned)yo[j][6] | ((unsigned)yo[j][7] << 16);
        *reinterpret_cast<uint4*>(ry + 2 * x0) = w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2 * QPT; k++) {
        if (x0 + k < P.W) {
          if (OUT8) ry[x0 + k] = (uint8_t)yo[j][k];
          else reinterpret_cast<uint16_t*>(ry)[x0 + k] = (uint16_t)yo[j][k];
        }
      }
    }
  }
  if (C444) return;
  uint8_t* ru = P.out[1] + f * P.out_fp[1] + cy * P.out_ls[1];
  uint8_t* rv = P.out[2] + f * P.out_fp[2] + cy * P.out_ls[2];
  if (VEC && full && QPT == 4) {
    if (OUT8) {
      *reinterpret_cast<unsigned*>(ru + cx0) =
          (unsigned)uo[0] | ((unsigned)uo[1] << 8) | ((unsigned)uo[2] << 16) | ((unsigned)uo[3] << 24);
      *reinterpret_cast<unsigned*>(rv + cx0) =
          (unsigned)vo[0] | ((unsigned)vo[1] << 8) | ((unsigned)vo[2] << 16) | ((unsigned)vo[3] << 24);
    } else {
      uint2 a, b;
      a.x = (unsigned)uo[0] | ((unsigned)uo[1] << 16);
      a.y = (unsigned)uo[2] | ((unsigned)uo[3] << 16);
      b.x = (unsigned)vo[0] | ((unsigned)vo[1] << 16);
      b.y = (unsigned)vo[2] | ((unsigned)vo[3] << 16);
      *reinterpret_cast<uint2*>(ru + 2 * cx0) = a;
      *reinterpret_cast<uint2*>(rv + 2 * cx0) = b;
    }
  } else {
#pragma unroll
    for (int k = 0; k < QPT; k++) {
      if (cx0 + k < cw) {
        if (OUT8) {
          ru[cx0 + k] = (uint8_t)uo[k];
          rv[cx0 + k] = (uint8_t)vo[k];
        } else {
          reinterpret_cast<uint16_t*>(ru)[cx0 + k] = (uint16_t)uo[k];
          reinterpret_cast<uint16_t*>(rv)[cx0 + k] = (uint16_t)vo[k];
        }
      }
    }
  }
  };
  // DYN (dynamic peak detection, one frame per launch): the frame's curve
  // constants come from the record the peak launches wrote on the device
  // (P0.cv), not from the launch parameters
  KParams P = P0;
  if (DYN) apply_curve(P, *P0.cv);
  if (LPX) X = lpx_consts(P, P.x_peak, P.x_avg);
  const long long lb = xcd_remap(blockIdx.x, gridDim.x);
  const long long item = lb * 256 + threadIdx.x;
  if (item >= P.total) return;
  const int gx = (int)(item % P.ngx);
  const long long t = item / P.ngx;
  body(P, (int)(t / P.ch), (int)(t % P.ch), (gx + P.gx0) * QPT);
}


// Debug/parity kernel: float RGB of frame 0 after stage STAGE, one thread per
// pixel, generic (unvectorised) sample access.
template <int STAGE>
__global__ __launch_bounds__(256) void k_debug(const KParams P, float* out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long npx = (long long)P.W * P.H;
  if (i >= npx) return;
  const int x = (int)(i % P.W), y = (int)(i / P.W);
  const int cw = P.cw, ch = P.ch;
  auto hpass = [&](int plane, int cyy) -> float {
    const uint8_t* row = P.in[plane] + edge(P, cyy, ch) * P.in_ls[plane];
    const int k = x >> 1;
    const float a = (float)(ld16(row, edge(P, k, cw)) & (int)P.in_mask) * P.c_scale + P.c_off;
    if (!(x & 1)) return a;
    const float b = (float)(ld16(row, edge(P, k + 1, cw)) & (int)P.in_mask) * P.c_scale + P.c_off;
    return 0.5f * a + 0.5f * b;
  };
  auto up = [&](int plane) -> float {
    const int m = y >> 1;
    if (!(y & 1)) return 0.25f * hpass(plane, m - 1) + 0.75f * hpass(plane, m);
    return 0.75f * hpass(plane, m) + 0.25f * hpass(plane, m + 1);
  };
  const float cb = up(1), cr = up(2);
  const int ycode = ld16(P.in[0] + y * P.in_ls[0], x) & (int)P.in_mask;
  const float yv = (float)ycode * P.y_scale + P.y_off;
  float r, g, b;
  if (P.pipe == PIPE_LIBPLACEBO) {   // the exact path (h2s_lpx.h), as k_process<..., LPX>
    auto hpd = [&](int plane, int cyy) -> double {
      const uint8_t* row = P.in[plane] + edge(P, cyy, ch) * P.in_ls[plane];
      const int k = x >> 1;
      const double a = lpx_chroma(P, ld16(row, edge(P, k, cw)) & (int)P.in_mask);
      if (!(x & 1)) return a;
      return 0.5 * (a + lpx_chroma(P, ld16(row, edge(P, k + 1, cw)) & (int)P.in_mask));
    };
    auto upd = [&](int plane) -> double {
      const int m = y >> 1;
      if (!(y & 1)) return 0.25 * hpd(plane, m - 1) + 0.75 * hpd(plane, m);
      return 0.75 * hpd(plane, m) + 0.25 * hpd(plane, m + 1);
    };
    const LpX X = lpx_consts(P, P.x_peak, P.x_avg);
    lpx_chain<STAGE < 5 ? STAGE : 4>(P, X, lpx_luma(P, ycode), upd(1), upd(2), x, y, r, g, b);
  } else {
    chain_px<STAGE < 5 ? STAGE : 4>(P, yv, cb, cr, r, g, b, lp_qoff(P, x, y));
  }
  if (STAGE == 5) {  // S6 quantiser inputs (oracle px_yuv)
    r = clamp01(r), g = clamp01(g), b = clamp01(b);
    const float Y = P.k709[0] * r + P.k709[1] * g + P.k709[2] * b;
    const float cbp = P.kcb[0] * r + P.kcb[1] * g + P.kcb[2] * b;
    const float crp = P.kcr[0] * r + P.kcr[1] * g + P.kcr[2] * b;
    r = (16.0f + 219.0f * Y) * P.qscale, g = 224.0f * P.qscale * cbp, b = 224.0f * P.qscale * crp;
  }
  out[i] = r;
  out[npx + i] = g;
  out[2 * npx + i] = b;
}

// BICUBIC chroma decimation (second pass): one thread per output chroma
// sample of one frame; separable taps (oracle process_frame_bicubic order:
// horizontal 7-tap sums per luma row, then the vertical 8-tap sum)
struct ChromaTaps {
  float wx[7], wy[8];
};

template <bool OUT8>
__global__ __launch_bounds__(256) void k_chroma_bicubic(const KParams P, const ChromaTaps T) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P.cw * P.ch) return;
  const int k = i % P.cw, m = i / P.cw;
  float su = 0.0f, sv = 0.0f;
  for (int j = 0; j < 8; j++) {
    const int y = min(max(2 * m - 3 + j, 0), P.H - 1);
    const float2* row = P.chr444 + (long long)y * P.W;
    float hu = 0.0f, hv = 0.0f;
#pragma unroll
    for (int t = 0; t < 7; t++) {
      const float2 c = row[min(max(2 * k - 3 + t, 0), P.W - 1)];
      hu += T.wx[t] * c.x;
      hv += T.wx[t] * c.y;
    }
    su += T.wy[j] * hu;
    sv += T.wy[j] * hv;
  }
  const float co = P.dither ? dither_off(k, m) : 0.5f;
  const int u = expand_code(P, quant_o((128.0f + 224.0f * su) * P.qscale, co, P.qmax));
  const int v = expand_code(P, quant_o((128.0f + 224.0f * sv) * P.qscale, co, P.qmax));
  uint8_t* ru = P.out[1] + m * P.out_ls[1];
  uint8_t* rv = P.out[2] + m * P.out_ls[2];
  if (OUT8) {
    ru[k] = (uint8_t)u, rv[k] = (uint8_t)v;
  } else {
    reinterpret_cast<uint16_t*>(ru)[k] = (uint16_t)u;
    reinterpret_cast<uint16_t*>(rv)[k] = (uint16_t)v;
  }
}

// ---- host-side launchers (called from h2s_api.hip) ----------------------
hipError_t launch_process(const KParams& P, bool vec, bool out8, hipStream_t s) {
  constexpr int QPT = 4;
  const long long nb = (P.total + 255) / 256;
  if (nb == 0) return hipSuccess;
  dim3 grid((unsigned)nb), block(256);
  if (P.pipe == PIPE_LIBPLACEBO) {   // the libplacebo branch's exact path (h2s_lpx.h)
    if (P.cv) {
      if (out8) hipLaunchKernelGGL((k_process<QPT, false, true, false, true, true>), grid, block, 0, s, P);
      else hipLaunchKernelGGL((k_process<QPT, false, false, false, true, true>), grid, block, 0, s, P);
    } else if (vec) {
      if (out8) hipLaunchKernelGGL((k_process<QPT, true, true, false, false, true>), grid, block, 0, s, P);
      else hipLaunchKernelGGL((k_process<QPT, true, false, false, false, true>), grid, block, 0, s, P);
    } else {
      if (out8) hipLaunchKernelGGL((k_process<QPT, false, true, false, false, true>), grid, block, 0, s, P);
      else hipLaunchKernelGGL((k_process<QPT, false, false, false, false, true>), grid, block, 0, s, P);
    }
    return hipGetLastError();
  }
  if (P.cv) {   // dynamic peak: the frame's curve record on the device
    if (out8) hipLaunchKernelGGL((k_process<QPT, false, true, false, true>), grid, block, 0, s, P);
    else hipLaunchKernelGGL((k_process<QPT, false, false, false, true>), grid, block, 0, s, P);
  } else if (vec) {
    if (out8) hipLaunchKernelGGL((k_process<QPT, true, true>), grid, block, 0, s, P);
    else hipLaunchKernelGGL((k_process<QPT, true, false>), grid, block, 0, s, P);
  } else {
    if (out8) hipLaunchKernelGGL((k_process<QPT, false, true>), grid, block, 0, s, P);
    else hipLaunchKernelGGL((k_process<QPT, false, false>), grid, block, 0, s, P);
  }
  return hipGetLastError();
}

hipError_t launch_debug(const KParams& P, int stage, float* out, hipStream_t s) {
  const long long npx = (long long)P.W * P.H;
  dim3 grid((unsigned)((npx + 255) / 256)), block(256);
  switch (stage) {
    case 1: hipLaunchKernelGGL((k_debug<1>), grid, block, 0, s, P, out); break;
    case 2: hipLaunchKernelGGL((k_debug<2>), grid, block, 0, s, P, out); break;
    case 3: hipLaunchKernelGGL((k_debug<3>), grid, block, 0, s, P, out); break;
    case 4: hipLaunchKernelGGL((k_debug<4>), grid, block, 0, s, P, out); break;
    default: hipLaunchKernelGGL((k_debug<5>), grid, block, 0, s, P, out); break;
  }
  return hipGetLastError();
}

// BICUBIC chroma, pass 1 on the generic kernel: k_process<C444> (luma +
// per-pixel chroma) over the launch's column groups (P.gx0, P.ngx)
hipError_t launch_process_c444(const KParams& P, bool out8, hipStream_t s) {
  constexpr int QPT = 4;
  const long long nb = (P.total + 255) / 256;
  if (nb == 0) return hipSuccess;
  if (P.pipe == PIPE_LIBPLACEBO) {   // the libplacebo branch's exact path (h2s_lpx.h)
    if (P.cv) {
      if (out8) hipLaunchKernelGGL((k_process<QPT, false, true, true, true, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
      else hipLaunchKernelGGL((k_process<QPT, false, false, true, true, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
    } else if (out8) {
      hipLaunchKernelGGL((k_process<QPT, false, true, true, false, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
    } else {
      hipLaunchKernelGGL((k_process<QPT, false, false, true, false, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
    }
    return hipGetLastError();
  }
  if (P.cv) {   // dynamic peak: the frame's curve record on the device
    if (out8) hipLaunchKernelGGL((k_process<QPT, false, true, true, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
    else hipLaunchKernelGGL((k_process<QPT, false, false, true, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
  } else if (out8) {
    hipLaunchKernelGGL((k_process<QPT, false, true, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
  } else {
    hipLaunchKernelGGL((k_process<QPT, false, false, true>), dim3((unsigned)nb), dim3(256), 0, s, P);
  }
  return hipGetLastError();
}

// BICUBIC chroma, pass 2: the decimation of one frame's chr444
hipError_t launch_chroma_bicubic(const KParams& P, const float* wx7, const float* wy8, bool out8, hipStream_t s) {
  ChromaTaps T;
  for (int i = 0; i < 7; i++) T.wx[i] = wx7[i];
  for (int j = 0; j < 8; j++) T.wy[j] = wy8[j];
  const unsigned nc = (unsigned)(((long long)P.cw * P.ch + 255) / 256);
  if (out8) hipLaunchKernelGGL((k_chroma_bicubic<true>), dim3(nc), dim3(256), 0, s, P, T);
  else hipLaunchKernelGGL((k_chroma_bicubic<false>), dim3(nc), dim3(256), 0, s, P, T);
  return hipGetLastError();
}

// ---- dynamic peak statistics (params.peak_detect, BT.2390) -----------------
// Per frame, the maximum and the sum of the PQ-encoded max(R,G,B) of every
// pixel (libplacebo peak detection, src/utils.py:448; PARITY UNPINNED: no
// libplacebo here, model in DESIGN.md).  PQ sources: PQ(max(EOTF(E))) ==
// clamp(max(E), 0, 1) exactly, so no transcendental is needed.  Chroma is
// taken nearest (the statistic is an estimate).  grid = (M.nblocks, frames);
// partial[f * M.nblocks + b] = (max, sum) over block b's rows / chunks
// one pixel's PQ-domain max(R,G,B) from its integer codes (nearest chroma)
template <int TRC>
__device__ __forceinline__ float peak_px(const KParams& P, unsigned yc, unsigned uc, unsigned vc) {
  yc &= P.in_mask, uc &= P.in_mask, vc &= P.in_mask;
  const float Y = (float)yc * P.y_scale + P.y_off;
  const float cb = (float)uc * P.c_scale + P.c_off, cr = (float)vc * P.c_scale + P.c_off;
  const float er = Y + P.m_rcr * cr, eg = Y + P.m_gcb * cb + P.m_gcr * cr, eb = Y + P.m_bcb * cb;
  if (TRC == 0) return clamp01(fmaxf(fmaxf(er, eg), eb));
  const float r = hlg_inv_oetf(er), g = hlg_inv_oetf(eg), bl = hlg_inv_oetf(eb);
  const float ys = 0.2627f * r + 0.6780f * g + 0.0593f * bl;
  const float w = ys > 0.0f ? P.lin_scale * apow(ys, 0.2f) : 0.0f;
  return clamp01(pq_encode(fmaxf(fmaxf(r, g), bl) * w * P.npl_1e4));
}

// percentile model (pd_percentile < 100; PARITY UNPINNED):
// a PEAK_BINS-bin histogram of the per-pixel PQ(max R,G,B) per frame; the
// percentile is interpolated inside its bin by k_peak_frame (oracle_peak_stats)
// a thread's run of equal bins, added to the LDS histogram once per run: on
// smooth content neighbouring pixels share a bin, and one LDS atomic per pixel
// had all 64 lanes of a wave serialise on one address; the
// counts are the same, only the number of atomics changes
struct HistRun {
  int bin = -1;
  unsigned n = 0;
  __device__ __forceinline__ void add(unsigned* lh, float m) {
    const int b = min((int)(m * (float)PEAK_BINS), PEAK_BINS - 1);
    if (b != bin) {
      if (n) atomicAdd(&lh[bin], n);
      bin = b, n = 0;
    }
    n++;
  }
  // n values of bin b (a whole quad-form unit in one step)
  __device__ __forceinline__ void add_n(unsigned* lh, int b, unsigned k) {
    if (b != bin) {
      if (n) atomicAdd(&lh[bin], n);
      bin = b, n = 0;
    }
    n += k;
  }
  __device__ __forceinline__ void flush(unsigned* lh) {
    if (n) atomicAdd(&lh[bin], n);
    n = 0;
  }
};
__device__ __forceinline__ void hist_flush(const unsigned* lh, unsigned* hist) {
  __syncthreads();
  for (int i = threadIdx.x; i < PEAK_BINS; i += 256)
    if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

// block (max, sum) reduction; thread 0 writes the record
__device__ __forceinline__ void peak_reduce(float mx, float sm, float2* out) {
  __shared__ float smx[256], ssm[256];
  smx[threadIdx.x] = mx, ssm[threadIdx.x] = sm;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + o]);
      ssm[threadIdx.x] += ssm[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = make_float2(smx[0], ssm[0]);
}

// ---- dynamic peak: per-frame statistic and curve records on the device ----
// One frame's (PQ peak measurement, average PQ) from its nblocks partial
// (max, sum) records and, for pd_percentile < 100, the percentile from the
// frame's histogram: the first bin whose cumulative count reaches pct % of
// the pixels, interpolated linearly inside it, capped at the frame maximum
// (oracle_peak_stats).  Wave-level reductions and scans (no LDS tree): the
// records fold in a fixed pairwise order in double (deterministic, so sharded
// and sequential statistics stay bit-identical), the counts are integers (a
// u32 scan equals a serial accumulation exactly).  The histogram is left
// zeroed for the next call.  256 threads.
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ void peak_frame_fold(const float2* partial, unsigned* hist, const PeakModel& M, double2* fstat, int f) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  __shared__ double s_sum[4];
  __shared__ float s_mx[4];
  __shared__ unsigned s_wtot[4];
  __shared__ int s_bin;
  static_assert(PEAK_BLOCKS_MAX <= 256, "one partial record per thread");
  const float2 rec = t < M.nblocks ? partial[(size_t)f * M.nblocks + t] : make_float2(0.0f, 0.0f);
  const double ws = wave_sum_d((double)rec.y);
  const float wm = wave_max_f(rec.x);
  if (lane == 0) s_sum[w] = ws, s_mx[w] = wm;
  if (t == 0) s_bin = PEAK_BINS;
  unsigned cnt[4] = {0u, 0u, 0u, 0u}, incl = 0u;
  if (M.pct) {
    static_assert(PEAK_BINS == 4 * 256, "four bins per thread");
    uint4* h = reinterpret_cast<uint4*>(hist + (size_t)f * PEAK_BINS);
    const uint4 c = h[t];
    h[t] = make_uint4(0u, 0u, 0u, 0u);
    cnt[0] = c.x, cnt[1] = c.y, cnt[2] = c.z, cnt[3] = c.w;
    incl = c.x + c.y + c.z + c.w;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {   // inclusive scan within the wave
      const unsigned v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) s_wtot[w] = incl;
  }
  __syncthreads();
  const double sum = (s_sum[0] + s_sum[1]) + (s_sum[2] + s_sum[3]);
  const double mx = (double)fmaxf(fmaxf(s_mx[0], s_mx[1]), fmaxf(s_mx[2], s_mx[3]));
  if (M.pct) {
    unsigned before = 0u, n = 0u;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      before += k < w ? s_wtot[k] : 0u;
      n += s_wtot[k];
    }
    const double target = M.percentile / 100.0 * (double)n;
    double cum = (double)(before + incl - (cnt[0] + cnt[1] + cnt[2] + cnt[3]));
    int mine = PEAK_BINS;
    double cum_at = 0.0;
    for (int k = 0; k < 4; k++) {
      if (mine == PEAK_BINS && cnt[k] && cum + cnt[k] >= target) mine = 4 * t + k, cum_at = cum;
      cum += cnt[k];
    }
    if (mine < PEAK_BINS) atomicMin(&s_bin, mine);
    __syncthreads();
    if (mine < PEAK_BINS && mine == s_bin) {   // the owner of the first bin
      const double v = (mine + (target - cum_at) / cnt[mine & 3]) / PEAK_BINS;
      fstat[f] = make_double2(v < mx ? v : mx, sum / M.npx);
    } else if (t == 0 && s_bin == PEAK_BINS) {
      fstat[f] = make_double2(mx, sum / M.npx);
    }
  } else if (t == 0) {
    fstat[f] = make_double2(mx, sum / M.npx);
  }
}

// The IIR over n frames in order (thread 0, from the state the previous calls
// left in *st), then each frame's peak and curve record in parallel.
// out = null: the state only.  Every thread of the block calls it.  The
// frames' statistics are staged through LDS, PEAK_IIR_CHUNK at a time, so
// the serial recurrence reads LDS instead of making a global round trip per
// frame (its loads could not be hoisted past the stores of the smoothed
// values: finish 20.8 -> see DESIGN.md §4.6)
constexpr int PEAK_IIR_CHUNK = 1024;
__device__ void peak_curves_body(double2* fstat, int n, const PeakModel& M, PeakState* st, CurveConsts* out) {
  const int t = threadIdx.x;
  __shared__ double2 s_f[PEAK_IIR_CHUNK];
  __shared__ PeakState s_st;
  if (t == 0) s_st = *st;
  for (int c0 = 0; c0 < n; c0 += PEAK_IIR_CHUNK) {
    const int cn = n - c0 < PEAK_IIR_CHUNK ? n - c0 : PEAK_IIR_CHUNK;
    __syncthreads();
    for (int f = t; f < cn; f += blockDim.x) s_f[f] = fstat[c0 + f];
    __syncthreads();
    if (t == 0) {
      PeakState s = s_st;
      for (int f = 0; f < cn; f++) {
        peak_iir_step(&s, M, s_f[f].x, s_f[f].y);
        s_f[f] = make_double2(s.max, s.avg);   // the smoothed values frame f's curve uses
      }
      s_st = s;
    }
    __syncthreads();
    for (int f = t; f < cn; f += blockDim.x) {
      fstat[c0 + f] = s_f[f];
      const double pk = peak_of(M, s_f[f].x);
      if (c0 + f == n - 1) s_st.peak = pk;    // the state's peak: the last frame's (its smoothed max)
      if (out) curve_for_peak(M, pk, s_f[f].y, &out[c0 + f]);
    }
  }
  __syncthreads();
  if (t == 0) *st = s_st;
}

// k_peak_finish: one block per frame folds that frame's records (and clears
// its histogram for the next call); the last frame to finish (a device-scope
// counter after a release fence: one per frame, so the fences stay few) runs
// the IIR and the curve records for all of the launch's frames.  PeakTail
// (h2s_peak.h) names the buffers; the counter is zeroed by the statistics
// launch queued before every finish launch (so an aborted launch cannot
// leave it stale) and left zero.
__global__ __launch_bounds__(256) void k_peak_finish(const float2* partial, const PeakTail T) {
  const int f = blockIdx.x;
  __shared__ int s_last;
  peak_frame_fold(partial, T.hist, T.M, T.fstat, f);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();   // fstat[f] and the cleared histogram, device-wide
    s_last = atomicAdd(T.done, 1u) == (unsigned)T.nframes - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  if (threadIdx.x == 0) *T.done = 0u;
  if (T.st) peak_curves_body(T.fstat, T.nframes, T.M, T.st, T.out);
}

// generic form: any width / alignment, 2-byte loads
template <int TRC, bool HIST>
__global__ __launch_bounds__(256) void k_peak_stats(const KParams P, float2* partial, const PeakTail T) {
  __shared__ unsigned lh[HIST ? PEAK_BINS : 1];
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *T.done = 0u;   // k_peak_finish's counter (stream-ordered)
  if (HIST)
    for (int i = threadIdx.x; i < PEAK_BINS; i += 256) lh[i] = 0;
  if (HIST) __syncthreads();
  const int f = blockIdx.y, b = blockIdx.x;
  float mx = 0.0f, sm = 0.0f;
  HistRun run;
  for (int y = b; y < P.H; y += gridDim.x) {
    const uint16_t* yr = reinterpret_cast<const uint16_t*>(P.in[0] + f * P.in_fp[0] + y * P.in_ls[0]);
    const uint16_t* ur = reinterpret_cast<const uint16_t*>(P.in[1] + f * P.in_fp[1] + (y >> 1) * P.in_ls[1]);
    const uint16_t* vr = reinterpret_cast<const uint16_t*>(P.in[2] + f * P.in_fp[2] + (y >> 1) * P.in_ls[2]);
    float rs = 0.0f;
    for (int x = threadIdx.x; x < P.W; x += blockDim.x) {
      const float m = peak_px<TRC>(P, yr[x], ur[x >> 1], vr[x >> 1]);
      mx = fmaxf(mx, m);
      rs += m;
      if (HIST) run.add(lh, m);
    }
    sm += rs;
  }
  if (HIST) run.flush(lh);
  if (HIST) hist_flush(lh, T.hist + (size_t)f * PEAK_BINS);
  peak_reduce(mx, sm, &partial[f * gridDim.x + b]);
}

// streaming form (W % 8 == 0, 16-byte luma / 8-byte chroma alignment): each
// thread takes 8-pixel row chunks (one 16-byte luma load, one 8-byte load per
// chroma plane), four chunks' loads in flight.  The round-5 default; the A/B
// reference of the quad form below (H2S_OPT_TEST_PEAK_FORM 1) and the form
// for HLG input
#ifndef H2S_PEAK_INFLIGHT
#define H2S_PEAK_INFLIGHT 4
#endif
template <int TRC, bool HIST>
__global__ __launch_bounds__(256) void k_peak_stats_v(const KParams P, float2* partial, const PeakTail T) {
  __shared__ unsigned lh[HIST ? PEAK_BINS : 1];
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *T.done = 0u;   // k_peak_finish's counter (stream-ordered)
  if (HIST)
    for (int i = threadIdx.x; i < PEAK_BINS; i += 256) lh[i] = 0;
  if (HIST) __syncthreads();
  const int f = blockIdx.y;
  const int cpr = P.W >> 3;                       // chunks per row
  const int nch = P.H * cpr, stride = gridDim.x * 256;
  const uint8_t* y0 = P.in[0] + f * P.in_fp[0];
  const uint8_t* u0 = P.in[1] + f * P.in_fp[1];
  const uint8_t* v0 = P.in[2] + f * P.in_fp[2];
  float mx = 0.0f, sm = 0.0f;
  HistRun run;
  struct Chunk {
    uint4 ya;
    uint2 ua, va;
  };
  auto load = [&](int i, Chunk& c) {
    const int r = i / cpr, cx = i - r * cpr;
    c.ya = reinterpret_cast<const uint4*>(y0 + r * P.in_ls[0])[cx];
    c.ua = reinterpret_cast<const uint2*>(u0 + (r >> 1) * P.in_ls[1])[cx];
    c.va = reinterpret_cast<const uint2*>(v0 + (r >> 1) * P.in_ls[2])[cx];
  };
  auto fold = [&](const Chunk& c) {
    const unsigned uu[4] = {c.ua.x & 0xffff, c.ua.x >> 16, c.ua.y & 0xffff, c.ua.y >> 16};
    const unsigned vv[4] = {c.va.x & 0xffff, c.va.x >> 16, c.va.y & 0xffff, c.va.y >> 16};
    const unsigned yy[8] = {c.ya.x & 0xffff, c.ya.x >> 16, c.ya.y & 0xffff, c.ya.y >> 16,
                            c.ya.z & 0xffff, c.ya.z >> 16, c.ya.w & 0xffff, c.ya.w >> 16};
    float rs = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const float m = peak_px<TRC>(P, yy[k], uu[k >> 1], vv[k >> 1]);
      mx = fmaxf(mx, m);
      rs += m;
      if (HIST) run.add(lh, m);
    }
    sm += rs;
  };
  int i = blockIdx.x * 256 + threadIdx.x;
  for (; i + (H2S_PEAK_INFLIGHT - 1) * stride < nch; i += H2S_PEAK_INFLIGHT * stride) {
    Chunk c[H2S_PEAK_INFLIGHT];
#pragma unroll
    for (int k = 0; k < H2S_PEAK_INFLIGHT; k++) load(i + k * stride, c[k]);
#pragma unroll
    for (int k = 0; k < H2S_PEAK_INFLIGHT; k++) fold(c[k]);
  }
  for (; i < nch; i += stride) {
    Chunk c;
    load(i, c);
    fold(c);
  }
  if (HIST) run.flush(lh);
  if (HIST) hist_flush(lh, T.hist + (size_t)f * PEAK_BINS);
  peak_reduce(mx, sm, &partial[f * gridDim.x + blockIdx.x]);
}

// quad form, the default for PQ input (W % 16 == 0, 16-byte rows; VERDICT
// r05 item 4): a thread's unit is 32 pixels -- 16 columns of a luma row pair
// and their 8 chroma samples -- read as six 16-byte loads (no chroma row read
// twice), two units' loads in flight.  PQ(max EOTF(R'G'B')) = clamp(max E):
// the chroma terms are maximised once per chroma sample (with Y's offset:
// d = y_off + max(a_rv v, a_gu u + a_gv v, a_bu u)) and each pixel is one FMA
// clamped to [0, 1] (E = code ys + d).  The histogram (pd_percentile < 100)
// takes a whole unit in one run step when the unit's smallest and largest
// values share a bin (bin() is monotonic: 55 % of the website frame's units);
// a unit that spans bins -- on the bench content 94 % of units span 8 or more
//  -- adds each value with its own LDS atomic, no run
// bookkeeping, the bin index floor(1024 m) unclamped into a 1025th entry (m =
// 1 exactly) folded into the last bin before the flush.  Every sum runs in a fixed
// order within the frame (unit by unit, 32 pixels row by row), so sharded
// and sequential statistics stay bit-identical.
template <bool HIST, int INF = 2>   // INF: units whose loads are in flight (4: A/B, H2S_OPT_TEST_PEAK_FORM 2)
__global__ __launch_bounds__(256) void k_peak_stats_q(const KParams P, float2* partial, const PeakTail T) {
  __shared__ unsigned lh[HIST ? PEAK_BINS + 1 : 1];   // + the bin of m = 1 exactly, folded into the last at the end
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *T.done = 0u;   // k_peak_finish's counter (stream-ordered)
  if (HIST)
    for (int i = threadIdx.x; i <= PEAK_BINS; i += 256) lh[i] = 0;
  if (HIST) __syncthreads();
  const int f = blockIdx.y;
  const int cpr = P.W >> 4, nch = (P.H >> 1) * cpr, stride = gridDim.x * 256;
  const uint8_t* y0 = P.in[0] + f * P.in_fp[0];
  const uint8_t* u0 = P.in[1] + f * P.in_fp[1];
  const uint8_t* v0 = P.in[2] + f * P.in_fp[2];
  const unsigned m2 = P.in_mask | (P.in_mask << 16);
  const float ys = P.y_scale, yo = P.y_off, cs = P.c_scale, co = P.c_off;
  float mx = 0.0f, sm = 0.0f;
  HistRun run;
  struct Unit {
    uint4 u, v, y0a, y0b, y1a, y1b;
  };
  auto load = [&](int i, Unit& q) {
    const int r = i / cpr, cx = i - r * cpr;
    q.u = *reinterpret_cast<const uint4*>(u0 + r * P.in_ls[1] + 16 * cx);
    q.v = *reinterpret_cast<const uint4*>(v0 + r * P.in_ls[2] + 16 * cx);
    const uint4* ya = reinterpret_cast<const uint4*>(y0 + 2 * r * P.in_ls[0] + 32 * cx);
    const uint4* yb = reinterpret_cast<const uint4*>(y0 + (2 * r + 1) * P.in_ls[0] + 32 * cx);
    q.y0a = ya[0], q.y0b = ya[1], q.y1a = yb[0], q.y1b = yb[1];
  };
  // the 32 values of a unit, in order, to fn(m)
  auto each = [&](const Unit& q, const float (&d)[8], auto&& fn) {
    const uint4 rows[4] = {q.y0a, q.y0b, q.y1a, q.y1b};
#pragma unroll
    for (int h = 0; h < 4; h++) {
      const unsigned w[4] = {rows[h].x & m2, rows[h].y & m2, rows[h].z & m2, rows[h].w & m2};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const unsigned code = (k & 1) ? w[k >> 1] >> 16 : w[k >> 1] & 0xffffu;
        fn(__builtin_amdgcn_fmed3f(fmaf((float)code, ys, d[4 * (h & 1) + (k >> 1)]), 0.0f, 1.0f));
      }
    }
  };
  auto fold = [&](const Unit& q) {
    const unsigned ua[4] = {q.u.x & m2, q.u.y & m2, q.u.z & m2, q.u.w & m2};
    const unsigned va[4] = {q.v.x & m2, q.v.y & m2, q.v.z & m2, q.v.w & m2};
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const float cb = fmaf((float)((j & 1) ? ua[j >> 1] >> 16 : ua[j >> 1] & 0xffffu), cs, co);
      const float cr = fmaf((float)((j & 1) ? va[j >> 1] >> 16 : va[j >> 1] & 0xffffu), cs, co);
      d[j] = yo + fmaxf(fmaxf(P.m_rcr * cr, fmaf(P.m_gcb, cb, P.m_gcr * cr)), P.m_bcb * cb);
    }
    float rs = 0.0f, umx = 0.0f, umn = 1.0f;
    each(q, d, [&](float m) {
      umx = fmaxf(umx, m);
      umn = fminf(umn, m);
      rs += m;
    });
    mx = fmaxf(mx, umx);
    sm += rs;
    if (HIST) {
      const int b0 = min((int)(umn * (float)PEAK_BINS), PEAK_BINS - 1);
      const int b1 = min((int)(umx * (float)PEAK_BINS), PEAK_BINS - 1);
      if (b0 == b1) {
        run.add_n(lh, b0, 32u);
      } else {
        each(q, d, [&](float m) { atomicAdd(&lh[(unsigned)(m * (float)PEAK_BINS)], 1u); });
      }
    }
  };
  int i = blockIdx.x * 256 + threadIdx.x;
  for (; i + (INF - 1) * stride < nch; i += INF * stride) {
    Unit q[INF];
#pragma unroll
    for (int k = 0; k < INF; k++) load(i + k * stride, q[k]);
#pragma unroll
    for (int k = 0; k < INF; k++) fold(q[k]);
  }
  for (; i < nch; i += stride) {
    Unit q;
    load(i, q);
    fold(q);
  }
  if (HIST) {
    run.flush(lh);
    __syncthreads();
    if (threadIdx.x == 0) lh[PEAK_BINS - 1] += lh[PEAK_BINS];
    hist_flush(lh, T.hist + (size_t)f * PEAK_BINS);
  }
  peak_reduce(mx, sm, &partial[f * gridDim.x + blockIdx.x]);
}

// the statistics of P's frames, then (k_peak_finish) their (measurement,
// average) in T.fstat and, T.st set, the smoothed state and curve records:
// two launches
hipError_t launch_peak_stats(const KParams& P, float2* partial, const PeakTail& T, hipStream_t s) {
  if (P.nframes <= 0) return hipSuccess;
  const dim3 grid(T.M.nblocks, P.nframes);
  auto al = [](long long v, int a) { return (v & (a - 1)) == 0; };
  auto planes_al = [&](int ya, int ca) {
    return al((long long)(uintptr_t)P.in[0], ya) && al(P.in_ls[0], ya) && al(P.in_fp[0], ya) &&
           al((long long)(uintptr_t)P.in[1], ca) && al(P.in_ls[1], ca) && al(P.in_fp[1], ca) &&
           al((long long)(uintptr_t)P.in[2], ca) && al(P.in_ls[2], ca) && al(P.in_fp[2], ca);
  };
  const bool vec = P.W % 8 == 0 && planes_al(16, 8);
  const bool quad = P.W % 16 == 0 && P.transfer == 0 && T.form != 1 && planes_al(16, 16);
#define H2S_PEAK_LAUNCH(HI)                                                                   \
  if (quad && T.form == 2)                                                                    \
    hipLaunchKernelGGL((k_peak_stats_q<HI, 4>), grid, dim3(256), 0, s, P, partial, T);        \
  else if (quad)                                                                              \
    hipLaunchKernelGGL((k_peak_stats_q<HI>), grid, dim3(256), 0, s, P, partial, T);           \
  else if (vec && P.transfer == 1)                                                            \
    hipLaunchKernelGGL((k_peak_stats_v<1, HI>), grid, dim3(256), 0, s, P, partial, T);        \
  else if (vec)                                                                               \
    hipLaunchKernelGGL((k_peak_stats_v<0, HI>), grid, dim3(256), 0, s, P, partial, T);        \
  else if (P.transfer == 1)                                                                   \
    hipLaunchKernelGGL((k_peak_stats<1, HI>), grid, dim3(256), 0, s, P, partial, T);          \
  else                                                                                        \
    hipLaunchKernelGGL((k_peak_stats<0, HI>), grid, dim3(256), 0, s, P, partial, T);
  if (T.M.pct) {
    H2S_PEAK_LAUNCH(true)
  } else {
    H2S_PEAK_LAUNCH(false)
  }
#undef H2S_PEAK_LAUNCH
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_peak_finish, dim3(P.nframes), dim3(256), 0, s, partial, T);
  return hipGetLastError();
}

// h2s_peak_feed: the IIR over caller-supplied statistics.  One block
void __global__ __launch_bounds__(64) k_peak_curves(double2* fstat, int n, const PeakModel M, PeakState* st,
                                                    CurveConsts* out) {
  peak_curves_body(fstat, n, M, st, out);
}

hipError_t launch_peak_curves(double2* fstat, int n, const PeakModel& M, PeakState* st, CurveConsts* out,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_peak_curves, dim3(1), dim3(64), 0, s, fstat, n, M, st, out);
  return hipGetLastError();
}

// The libplacebo branch's lut3d 8-bit table for the tile kernel: for every
// rgba8 code triple (r, g, b), lut3d's 8-bit output -- coordinate (q / 255)
// (N-1), tetrahedral blend, truncation -- in this translation unit's
// arithmetic (no FMA contraction: the oracle's lut3d_8bit order, as
// chain_px / lpx_chain), packed R | G << 8 | B << 16.  2^24 entries, 64 MiB;
// built once per lattice (h2s_api.hip ensure_lut8x)
// The entries are in bit-interleaved (Morton) order -- index bit 3k = r bit
// k, 3k+1 = g bit k, 3k+2 = b bit k -- so that a 128-byte line holds a 4 x 4
// x 2 block of codes (the order r | g << 8 | b << 16 measured up to 42 %
// slower on smooth content: profiles/r06/lp_table/, patch in
// profiles/r06/ab_patches/lp_tab_linear.patch)
__global__ __launch_bounds__(256) void k_build_lut8x(const KParams P, unsigned* out) {
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  unsigned cr = 0, cg = 0, cb = 0;
  for (int k = 0; k < 8; k++) {
    cr |= ((i >> (3 * k)) & 1u) << k;
    cg |= ((i >> (3 * k + 1)) & 1u) << k;
    cb |= ((i >> (3 * k + 2)) & 1u) << k;
  }
  const float sf = 1.0f / 255.0f;
  float r = (float)cr * sf, g = (float)cg * sf, b = (float)cb * sf;
  lut3d_tetra(P, r, g, b);
  const unsigned R = (unsigned)fminf(fmaxf(truncf(r * 255.0f), 0.0f), 255.0f);
  const unsigned G = (unsigned)fminf(fmaxf(truncf(g * 255.0f), 0.0f), 255.0f);
  const unsigned B = (unsigned)fminf(fmaxf(truncf(b * 255.0f), 0.0f), 255.0f);
  out[i] = R | (G << 8) | (B << 16);
}

hipError_t build_lut8x(const float4* lut, int n, unsigned* out, hipStream_t s) {
  KParams P{};
  P.lut = lut, P.lut_n = n, P.lut_sg = n, P.lut_sb = n * n, P.lut_max = (float)(n - 1);
  hipLaunchKernelGGL(k_build_lut8x, dim3((1u << 24) / 256), dim3(256), 0, s, P, out);
  return hipGetLastError();
}

// device libm_powf / libm_expf over n inputs (fn 0: powf(x, y), 1: expf(x)),
// for tests/test_libm_tables.py's bit-equality check against the libm the
// oracle links
__global__ void k_test_libm(int fn, const float* x, const float* y, float* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = fn == 0 ? libm_powf(x[i], y[i]) : libm_expf(x[i]);
}

}  // namespace h2s

// Private test entry (not part of the C-ABI, not declared in include/h2s.h):
// host arrays in and out, synchronous, on the current device.  Returns 0 or
// a negative HIP error.
extern "C" __attribute__((visibility("default"))) int h2stest_libm(int fn, const float* x, const float* y, float* out,
                                                                    int n) {
  if (n <= 0) return 0;
  float* d = nullptr;
  const size_t b = (size_t)n * sizeof(float);
  if (hipMalloc(&d, 3 * b) != hipSuccess) return -1;
  hipError_t e = hipMemcpy(d, x, b, hipMemcpyHostToDevice);
  if (e == hipSuccess && y) e = hipMemcpy(d + n, y, b, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(h2s::k_test_libm, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, d, d + n, d + 2 * n, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, d + 2 * n, b, hipMemcpyDeviceToHost);
  hipFree(d);
  return e == hipSuccess ? 0 : -(int)e;
}

// private test hook (not in include/h2s.h): the libplacebo branch's lut3d
// 8-bit table (k_build_lut8x) for a host lattice of n^3 R'G'B' records (3
// floats each, r fastest), copied back in the kernel's bit-interleaved
// order (2^24 u32).  For tests/test_gpu_parity.py's whole-table comparison
// with the oracle's lut3d 8-bit path.  Returns 0 or a negative HIP error.
extern "C" __attribute__((visibility("default"))) int h2stest_lut8x(const float* lut_rgb, int n, unsigned* out) {
  if (n < 2 || n > 256) return -1;
  const size_t nn = (size_t)n * n * n;
  std::vector<float4> l4(nn + 1, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
  for (size_t i = 0; i < nn; i++) l4[i] = make_float4(lut_rgb[3 * i], lut_rgb[3 * i + 1], lut_rgb[3 * i + 2], 0.0f);
  float4* dl = nullptr;
  unsigned* dt = nullptr;
  if (hipMalloc(&dl, l4.size() * sizeof(float4)) != hipSuccess) return -1;
  if (hipMalloc(&dt, sizeof(unsigned) << 24) != hipSuccess) {
    hipFree(dl);
    return -1;
  }
  hipError_t e = hipMemcpy(dl, l4.data(), l4.size() * sizeof(float4), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = h2s::build_lut8x(dl, n, dt, 0);
  if (e == hipSuccess) e = hipMemcpy(out, dt, sizeof(unsigned) << 24, hipMemcpyDeviceToHost);
  hipFree(dl);
  hipFree(dt);
  return e == hipSuccess ? 0 : -(int)e;
}
