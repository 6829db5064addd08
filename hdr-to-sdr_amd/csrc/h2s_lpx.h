// h2s_lpx.h — the libplacebo branch (src/utils.py:444-460) on the generic
// kernel: stages 1-3 as exact arithmetic (double precision from the integer
// codes), down to the 8-bit rgba download's pre-rounding value.
//
// The reference runs this branch's tone mapping in libplacebo's float32 GLSL
// on a Vulkan GPU, so no particular float32 evaluation is the reference; the
// oracle states the branch as exact arithmetic (oracle/h2s_oracle.c
// chain_lp_d) and this is the same statement on the device: same operation
// order, same constants, double pow / exp.  It is the branch's exact path
// (H2S_OPT_LP_EXACT) and serves whatever the tile kernel does not cover (the
// ragged columns, N > 177 lattices, BICUBIC two-pass).  The tile kernel's
// float32 form lands within its stated bound of these values
// (tests/lp_gate.py).  Stage 4 on (lut3d's 8-bit path on the integer codes,
// Y'CbCr) is the float arithmetic of h2s_device.h, as the oracle's.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>

#include "h2s_device.h"

namespace h2s {

// ST 2084 in double (normalised, 1 = 10000 nits): zimg's EOTF (denominator
// floored at FLT_MIN; past the pole +inf, as the float form) and the inverse
__device__ __forceinline__ double pqx_eotf(double e) {
  if (!(e > 0.0)) return 0.0;
  const double xp = pow(e, 1.0 / (double)PQ_M2);
  const double num = xp - (double)PQ_C1 > 0.0 ? xp - (double)PQ_C1 : 0.0;
  const double den = (double)PQ_C2 - (double)PQ_C3 * xp;
  const double v = pow(num / (den > (double)FLT_MIN ? den : (double)FLT_MIN), 1.0 / (double)PQ_M1);
  return v > (double)FLT_MAX ? __builtin_inf() : v;
}
__device__ __forceinline__ double pqx_encode(double y) {
  const double ym = pow(y > 0.0 ? y : 0.0, (double)PQ_M1);
  return pow(((double)PQ_C1 + (double)PQ_C2 * ym) / (1.0 + (double)PQ_C3 * ym), (double)PQ_M2);
}
// ARIB STD-B67 inverse OETF with the specification's constants
__device__ __forceinline__ double hlgx_inv_oetf(double x) {
  const double a = 0.17883277, b = 0.28466892, c = 0.55991073;
  x = x > 0.0 ? x : 0.0;
  return x <= 0.5 ? x * x / 3.0 : (exp((x - c) / a) + b) / 12.0;
}
__device__ __forceinline__ double hablex(double x) {
  const double a = 0.15, b = 0.50, c = 0.10, d = 0.20, e = 0.02, f = 0.30;
  return (x * (x * a + b * c) + d * e) / (x * (x * a + b) + d * f) - e / f;
}

// the branch's constants for a source peak (units of 100 nits) and average
// PQ level (spline knee; 0 = the default knee), oracle resolve / spline_setup
struct LpX {
  double tw, tb, out_scale, enc_a, enc_b, n_peak, npl;
  double src_min, src_max, max_lum, min_lum, ks, bp, bgain;
  double sp_smin, sp_smax, sp_dmin, sp_dmax, sp_kin, sp_kout, sp_pa, sp_pb, sp_qa, sp_qb, sp_qc;
  double tm_param;   // NaN: the curve's default
  int tonemap, ipt;
};

__device__ __forceinline__ LpX lpx_consts(const KParams& P, double peak, double avg_pq) {
  LpX X;
  X.tw = P.t_white, X.tb = P.t_black, X.npl = P.x_npl, X.tm_param = P.x_tm_param;
  X.tonemap = P.tonemap, X.ipt = P.lp_ipt;
  X.out_scale = 10000.0 / X.tw;
  const double lb = pow(X.tb / X.tw, 1.0 / 2.4);
  X.enc_a = pow(1.0 - lb, 2.4);
  X.enc_b = lb / (1.0 - lb);
  X.n_peak = peak * 100.0 / X.tw;
  X.src_min = pqx_encode(0.0);
  X.src_max = pqx_encode(peak * 100.0 / 10000.0);
  X.max_lum = (pqx_encode(X.tw / 10000.0) - X.src_min) / (X.src_max - X.src_min);
  X.min_lum = X.tb > 0.0 ? (pqx_encode(X.tb / 10000.0) - X.src_min) / (X.src_max - X.src_min) : 0.0;
  X.ks = (1.0 + P.knee_off) * X.max_lum - P.knee_off;
  X.bp = X.min_lum > 0.0 ? fmin(1.0 / X.min_lum, 4.0) : 4.0;
  X.bgain = X.max_lum < 1.0 ? 1.0 / (1.0 + X.min_lum / X.max_lum * pow(1.0 - X.max_lum, X.bp)) : 1.0;
  if (X.tonemap == 8) {   // spline_setup
    const double kad = 0.4, kmin = 0.1, kmax = 0.8, kdef = 0.4, st = 1.5, so = 0.2;
    auto smooth = [](double e0, double e1, double x) {
      double t = (x - e0) / (e1 - e0);
      t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
      return t * t * (3.0 - 2.0 * t);
    };
    const double contrast = X.tm_param != X.tm_param ? 0.5 : X.tm_param;
    const double smin = X.src_min, smax = X.src_max;
    const double dmin = pqx_encode(X.tb / 10000.0), dmax = pqx_encode(X.tw / 10000.0);
    double sk = avg_pq > 0.0 ? avg_pq : smin + (smax - smin) * kdef;
    const double lo = smin + (smax - smin) * kmin, hi = smin + (smax - smin) * kmax;
    sk = sk < lo ? lo : (sk > hi ? hi : sk);
    const double target = (sk - smin) / (smax - smin);
    const double adapted = dmin + (dmax - dmin) * target;
    const double tuning = 1.0 - smooth(kmax, kdef, target) * smooth(kmin, kdef, target);
    const double adaptation = kad + (1.0 - kad) * tuning;
    double dk = sk + (adapted - sk) * adaptation;
    dk = dk < dmin ? dmin : (dk > dmax ? dmax : dk);
    double ratio = st * (smax / dmax - 1.0);
    ratio = ratio < so ? so : (ratio > 1.0 + so ? 1.0 + so : ratio);
    const double slope = pow(pqx_eotf(dk) / pqx_eotf(sk), (1.0 - contrast) * ratio);
    const double in_min = smin - sk, in_max = smax - sk, out_min = dmin - dk, out_max = dmax - dk;
    X.sp_smin = smin, X.sp_smax = smax, X.sp_dmin = dmin, X.sp_dmax = dmax, X.sp_kin = sk, X.sp_kout = dk;
    X.sp_pa = (out_min - slope * in_min) / (in_min * in_min);
    X.sp_pb = slope;
    X.sp_qa = (slope * in_max - out_max) / (in_max * 2.0 * in_max * in_max);
    X.sp_qb = -3.0 * (slope * in_max - out_max) / (2.0 * in_max * in_max);
    X.sp_qc = slope;
  }
  return X;
}

// libplacebo's reinhard / hable / mobius in NORM units (oracle lp_norm_curve_d)
__device__ __forceinline__ double lpx_norm_curve(const LpX& X, double x) {
  const double pk = X.n_peak;
  x = x < 0.0 ? 0.0 : (x > pk ? pk : x);
  if (X.tonemap == 4) {
    const double ct = X.tm_param != X.tm_param ? 0.5 : X.tm_param;
    const double off = (1.0 - ct) / ct, scale = (pk + off) / pk;
    return scale * x / (x + off);
  }
  if (X.tonemap == 5) return hablex(x) / hablex(pk);
  const double j = X.tm_param != X.tm_param ? 0.3 : X.tm_param;
  if (x <= j) return x;
  const double a = -j * j * (pk - 1.0) / (j * j - 2.0 * j + pk);
  const double b = (j * j - 2.0 * j * pk + pk) / fmax(1e-6, pk - 1.0);
  return (b * b + 2.0 * b * j + j * j) / (b - a) * (x + a) / (x + b);
}

// BT.2390 / spline on a PQ-domain signal (oracle bt2390_pq_d / spline_pq_d)
__device__ __forceinline__ double lpx_bt2390(const LpX& X, double e1) {
  double e1n = (e1 - X.src_min) / (X.src_max - X.src_min);
  e1n = e1n != e1n ? 1.0 : (e1n < 0.0 ? 0.0 : (e1n > 1.0 ? 1.0 : e1n));
  const double ks = X.ks, ml = X.max_lum;
  double e2 = e1n;
  if (ks < 1.0 && e1n > ks) {
    const double t = (e1n - ks) / (1.0 - ks), t2 = t * t, t3 = t2 * t;
    e2 = (2.0 * t3 - 3.0 * t2 + 1.0) * ks + (t3 - 2.0 * t2 + t) * (1.0 - ks) + (-2.0 * t3 + 3.0 * t2) * ml;
  }
  if (X.min_lum > 0.0 && e2 < 1.0) {
    e2 += X.min_lum * pow(1.0 - e2, X.bp);
    e2 = X.bgain * (e2 - X.min_lum) + X.min_lum;
  }
  return e2 * (X.src_max - X.src_min) + X.src_min;
}
__device__ __forceinline__ double lpx_spline(const LpX& X, double e) {
  double x = e < X.sp_smin ? X.sp_smin : (e > X.sp_smax ? X.sp_smax : e);
  x -= X.sp_kin;
  double y = x > 0.0 ? ((X.sp_qa * x + X.sp_qb) * x + X.sp_qc) * x : (X.sp_pa * x + X.sp_pb) * x;
  y += X.sp_kout;
  return y < X.sp_dmin ? X.sp_dmin : (y > X.sp_dmax ? X.sp_dmax : y);
}
__device__ __forceinline__ double lpx_curve_pq(const LpX& X, double e) {
  if (X.tonemap == 7) return lpx_bt2390(X, e);
  if (X.tonemap == 8) return lpx_spline(X, e);
  return pqx_encode(lpx_norm_curve(X, pqx_eotf(e) * (10000.0 / X.tw)) * (X.tw / 10000.0));
}

// S2 of the branch (oracle tone_lp_d): the IPT form, or the max(R,G,B) gain;
// inputs capped at 1e6 npl in the IPT form and the NORM curves' gain
__device__ __forceinline__ void lpx_tone(const KParams& P, const LpX& X, double& r, double& g, double& b) {
  const bool capped = X.ipt || (X.tonemap >= 4 && X.tonemap <= 6);
  if (capped) r = fmin(r, 1e6), g = fmin(g, 1e6), b = fmin(b, 1e6);
  if (X.ipt) {
    const double s = X.npl / 10000.0, w0 = r * s, w1 = g * s, w2 = b * s;
    double q[3], l[3];
#pragma unroll
    for (int k = 0; k < 3; k++) q[k] = pqx_encode(P.ipt_r2l[3 * k] * w0 + P.ipt_r2l[3 * k + 1] * w1 + P.ipt_r2l[3 * k + 2] * w2);
    const double I = 0.4 * q[0] + 0.4 * q[1] + 0.2 * q[2];
    const double dI = lpx_curve_pq(X, I) - I;
#pragma unroll
    for (int k = 0; k < 3; k++) l[k] = pqx_eotf(q[k] + dI);
    const double os = X.out_scale;
    r = (P.ipt_l2r[0] * l[0] + P.ipt_l2r[1] * l[1] + P.ipt_l2r[2] * l[2]) * os;
    g = (P.ipt_l2r[3] * l[0] + P.ipt_l2r[4] * l[1] + P.ipt_l2r[5] * l[2]) * os;
    b = (P.ipt_l2r[6] * l[0] + P.ipt_l2r[7] * l[1] + P.ipt_l2r[8] * l[2]) * os;
    return;
  }
  double sig = r > g ? r : g;
  sig = sig > b ? sig : b;
  sig = sig > 1e-6 ? sig : 1e-6;
  double k;
  if (X.tonemap >= 4 && X.tonemap <= 6)
    k = lpx_norm_curve(X, sig * (X.npl / X.tw)) / sig;
  else
    k = pqx_eotf(lpx_curve_pq(X, pqx_encode(sig * (X.npl / 10000.0)))) * X.out_scale / sig;
  r *= k, g *= k, b *= k;
}

__device__ __forceinline__ double lpx_encode(const LpX& X, double x) {
  if (!(x > 0.0)) x = 0.0;
  return pow(x / X.enc_a, 1.0 / 2.4) - X.enc_b;
}

// one pixel of the branch from its exact Y', Cb, Cr (normalised, double):
// UPTO 1..3 = that stage's values, 4 = lut3d's 8-bit output / 255 (LUT on)
// or the encoded BT.709 R'G'B' clipped (LUT off); px, py: the pixel (dither)
template <int UPTO>
__device__ __forceinline__ void lpx_chain(const KParams& P, const LpX& X, double yv, double cb, double cr, int px,
                                          int py, float& ro, float& go, float& bo) {
  const double kr = 0.2627, kb = 0.0593, kg = 1.0 - kr - kb;
  const double er = yv + 2.0 * (1.0 - kr) * cr;
  const double eg = yv - 2.0 * kb * (1.0 - kb) / kg * cb - 2.0 * kr * (1.0 - kr) / kg * cr;
  const double eb = yv + 2.0 * (1.0 - kb) * cb;
  double r, g, b;
  if (P.transfer == 1) {
    r = hlgx_inv_oetf(er), g = hlgx_inv_oetf(eg), b = hlgx_inv_oetf(eb);
    const double ys = 0.2627 * r + 0.6780 * g + 0.0593 * b;
    const double w = ys > 0.0 ? 1000.0 / X.npl * pow(ys, 0.2) : 0.0;
    r *= w, g *= w, b *= w;
  } else {
    const double s = 10000.0 / X.npl;
    r = pqx_eotf(er) * s, g = pqx_eotf(eg) * s, b = pqx_eotf(eb) * s;
  }
  if (UPTO == 1) {
    ro = (float)r, go = (float)g, bo = (float)b;
    return;
  }
  lpx_tone(P, X, r, g, b);
  if (UPTO == 2) {
    ro = (float)r, go = (float)g, bo = (float)b;
    return;
  }
  if (P.lut_enabled) {
    const double e[3] = {lpx_encode(X, r), lpx_encode(X, g), lpx_encode(X, b)};
    if (UPTO == 3) {
      ro = (float)e[0], go = (float)e[1], bo = (float)e[2];
      return;
    }
    // the rgba8 download: floor(clamp01(v) qs + qo + offset), exactly
    const double off = (double)P.lp_qo + (P.lp_dith ? (double)bayer16(px, py) : 0.5);
    float q[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const double v = e[k] < 0.0 ? 0.0 : (e[k] > 1.0 ? 1.0 : e[k]);
      q[k] = (float)floor(v * (double)P.lp_qs + off) * (1.0f / 255.0f);
    }
    // vf_lut3d's 8-bit path on the codes (h2s_device.h lut3d_8bit after its rounding)
    float lr = q[0], lg = q[1], lb = q[2];
    lut3d_tetra(P, lr, lg, lb);
    const float sf = 1.0f / 255.0f;
    ro = fminf(fmaxf(truncf(lr * 255.0f), 0.0f), 255.0f) * sf;
    go = fminf(fmaxf(truncf(lg * 255.0f), 0.0f), 255.0f) * sf;
    bo = fminf(fmaxf(truncf(lb * 255.0f), 0.0f), 255.0f) * sf;
    return;
  }
  // LUT off: libplacebo's BT.2020 -> BT.709 matrix (tools/generate_lut.py:36-40), encode, clip
  const double m[9] = {1.6604910021, -0.5876411388, -0.0728498633, -0.1245504745, 1.1328998971,
                       -0.0083494226, -0.0181507634, -0.1005788980, 1.1187296614};
  double o[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const double v = lpx_encode(X, m[3 * k] * r + m[3 * k + 1] * g + m[3 * k + 2] * b);
    o[k] = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
  }
  ro = (float)o[0], go = (float)o[1], bo = (float)o[2];
}

// exact normalised samples from integer codes (zimg's limited-range
// conversion without its float rounding): luma (c - 16 s) / 219 s, chroma
// (c - 128 s) / 224 s, s = 2^(bits - 8)
__device__ __forceinline__ double lpx_luma(const KParams& P, int code) {
  return ((double)code - (double)(16 << P.x_sh)) / (double)(219 << P.x_sh);
}
__device__ __forceinline__ double lpx_chroma(const KParams& P, int code) {
  return ((double)code - (double)(128 << P.x_sh)) / (double)(224 << P.x_sh);
}

}  // namespace h2s
