// h2s_device.h — per-pixel chain for gfx950 (device code) and the launch
// parameter block shared by the kernels and the host launcher.
//
// Stage numbering follows the reference chain string (src/utils.py:38-42):
//   S1 zscale=t=linear:npl=100   S2 tonemap={tm}   S3 zscale=t=bt709
//   S4 lut3d=interp=tetrahedral  S6 (auto) scale->yuv420p  S7 eq=gamma
//   S8 (auto) scale->-pix_fmt (src/ffmpeg_command.py:355-360)
// The CPU statement each function must agree with is oracle/h2s_oracle.c.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "h2s_libm.h"

namespace h2s {

struct CurveConsts;

struct KParams {
  // geometry (luma W x H, chroma cw x ch, ngx groups of QPT chroma columns)
  int W, H, cw, ch, ngx;
  int nframes;
  long long total;  // nframes * ch * ngx work items
  const uint8_t* in[3];
  long long in_ls[3], in_fp[3];
  uint8_t* out[3];
  long long out_ls[3], out_fp[3];
  // S1: zimg depth conversion, BT.2020-NCL matrix, transfer
  float y_scale, y_off, c_scale, c_off;
  float m_rcr, m_gcb, m_gcr, m_bcb;
  float lin_scale;
  int transfer;  // h2s_transfer
  // S2: vf_tonemap
  int tonemap;  // h2s_tonemap
  int desat_on;
  float desat, lr, lg, lb;
  float lin_k;          // LINEAR: param/peak
  float gam_inv_peak, gam_inv_param, gam_low_k;  // GAMMA
  float clip_k;         // CLIP: param
  float hable_peak_inv; // HABLE: 1/hable(peak)
  float rein_p, rein_k; // REINHARD: param, (peak+param)/peak
  float mob_j, mob_a, mob_b, mob_k;  // MOBIUS
  float b_srcmin, b_range, b_inv_range, b_ks, b_inv_1mks, b_maxlum;  // BT2390
  float npl_1e4, e4_npl;  // npl/10000, 10000/npl
  // SPLINE (libplacebo, PQ domain): clip range, knee, toe P, shoulder Q, output range
  float sp_srcmin, sp_srcmax, sp_kin, sp_kout, sp_pa, sp_pb, sp_qa, sp_qb, sp_qc, sp_dmin, sp_dmax;
  float sp_contrast;
  double peak;            // resolved static source peak (units of 100 nits; host side)
  // libplacebo bt2390 black-point adaptation (min_lum = 0: off)
  float b_minlum, b_bp, b_gain;
  double t_black, t_white, knee_off;  // SDR target (nits) and BT.2390 knee offset (host side)
  // pipeline (h2s_pipeline, resolved to CPU_CHAIN or LIBPLACEBO)
  int pipe, rgba8;
  float enc_ainv, enc_b;  // libplacebo BT.1886 encode: (x * ainv)^(1/2.4) - b
  float enc_a;            // (the generic kernel divides by a, as the oracle)
  int lp_ipt;             // libplacebo branch: the curve on IPT-PQ intensity (h2s_lp_tone IPT)
  // libplacebo branch options (include/h2s.h ABI v3): rgba8 code =
  // floor(clamp01(v) lp_qs + lp_qo + (lp_dith ? bayer16(x, y) : 0.5));
  // in_mask: input code mask (0xFFFC: a 12-bit input through format=p010
  // with the two low bits dropped, h2s_lp_p010 TRUNCATE)
  float lp_qs, lp_qo;
  int lp_dith;
  unsigned in_mask;
  // peak_detect (host side): IIR period (frames), scene thresholds (% PQ),
  // percentile, minimum peak (units of 100 nits)
  double pd_smoothing, pd_scene_low, pd_scene_high, pd_percentile, pd_min;
  double ipt_r2l[9], ipt_l2r[9];  // BT.2020 RGB -> LMS (HPE), inverse (row-major)
  double ipt_npl, ipt_os, ipt_tw; // npl / 10000, 10000 / target white, target white / 10000 (double)
  // libplacebo reinhard / hable / mobius (scaling PL_HDR_NORM: 1 = target white)
  int lp_norm;                    // the libplacebo branch with one of them
  float n_peak, n_nw;             // source peak / white; npl / white (npl units -> NORM)
  float n_rein_off, n_rein_scale, n_hable_inv, n_mob_j, n_mob_a, n_mob_b, n_mob_scale;
  // S3/S4
  int lut_enabled, lut_n, lut_sg, lut_sb;
  float lut_max;
  const float4* lut;
  float m709[9];
  // S6..S8
  int qmax, shift_out;
  float qscale;
  int eq_identity;
  const uint16_t* eq_lut;
  int chroma_edge;        // S1 upsampler edge rule (chroma_edge_at)
  int lut_in16;           // S3 -> S4 as 16-bit R'G'B' (h2s_lut_input RGB48)
  int dither;             // ordered 8x8 dither at the 8-bit quantiser
  int expand_rep;         // S8 bit replication instead of a shift
  // Y'CbCr 709 rows
  float k709[3], kcb[3], kcr[3];
  int gx0;  // first column group this launch covers (tail launches)
  float2* chr444;         // BICUBIC: per-pixel (Cb, Cr) of one frame (two-pass path)
  // dynamic peak detection (one frame per launch): the frame's curve record,
  // written on the device by k_peak_curves; null: the constants above
  const CurveConsts* cv;
  // the libplacebo branch's exact path (h2s_lpx.h): source peak (units of 100
  // nits) and average PQ level (0: the default spline knee) its double
  // constants derive from, npl, tm_param (NaN: default), bits_in - 8
  double x_peak, x_avg, x_npl, x_tm_param;
  int x_sh;
};

constexpr int PIPE_CPU = 1, PIPE_LIBPLACEBO = 2;

// S1 chroma upsampler edge rule (enum h2s_chroma_edge; oracle edge()): the
// sample read at position i of an n-sample chroma row / column.  0 ZIMG: -1
// mirrors to 1, n folds to n-1; 1 REPLICATE: both sides repeat the last
// sample; 2 MIRROR: both sides mirror about it (n -> n-2)
__host__ __device__ __forceinline__ int chroma_edge_at(int i, int n, int mode) {
  if (i < 0) i = mode == 1 ? 0 : -i;
  if (i > n - 1) i = mode == 2 ? 2 * (n - 1) - i : n - 1;
  return i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
}

// Constants of the PQ-domain curves (BT.2390 / spline) in the fast kernel's
// folded form.  They are the only parameters that change from frame to frame
// under dynamic peak detection, so a launch can take one record per frame.
struct CurveConsts {
  float b_srcmin, b_range, b_inv_range, b_ks, b_inv_1mks, b_maxlum;  // BT.2390, HLG input
  float b_minlum, b_bp, b_gain;  // black-point adaptation (b_minlum = 0: off)
  // PQ-input forms that land directly on pq_z's table coordinate u = e*PQ_SEG + 1:
  // BT.2390: e1n = med3(e1*e1a + e1b), t = e1n*ta + tb, u = c3..c0 Horner (knee) or e1n*lr + lc
  float b_e1a, b_e1b, b_ta, b_tb, b_c3, b_c2, b_c1, b_c0, b_lr, b_lc, b_thr;
  float sp_srcmin, sp_srcmax, sp_kin, sp_kout, sp_pa, sp_pb, sp_qa, sp_qb, sp_qc, sp_dmin, sp_dmax;  // SPLINE
  // spline: u = Horner(x) with the coefficients and kout scaled by PQ_SEG, clamped to [umin, umax]
  float sp_qa_u, sp_qb_u, sp_qc_u, sp_pa_u, sp_pb_u, sp_k_u, sp_umin, sp_umax;
  // BT.2390 black-point adaptation on the table coordinate u = e2*R + C:
  // 1 - e2 = u*bk_a + bk_b; u' = gain*u + bk_c*(1 - e2)^bp + bk_d for e2 < 1
  float b_bk_a, b_bk_b, b_bk_c, b_bk_d;
  // libplacebo reinhard / hable / mobius in NORM units (1 = target white)
  float n_peak, n_rein_off, n_rein_scale, n_hable_inv, n_mob_j, n_mob_a, n_mob_b, n_mob_scale;
  // the frame's source peak (units of 100 nits) and smoothed average PQ level,
  // from which the generic kernel's exact libplacebo path (h2s_lpx.h) derives
  // its double constants
  double x_peak, x_avg;
};

// a frame's curve record over the generic kernel's constants (dynamic peak)
__device__ __forceinline__ void apply_curve(KParams& P, const CurveConsts& C) {
  P.b_srcmin = C.b_srcmin, P.b_range = C.b_range, P.b_inv_range = C.b_inv_range, P.b_ks = C.b_ks;
  P.b_inv_1mks = C.b_inv_1mks, P.b_maxlum = C.b_maxlum, P.b_minlum = C.b_minlum, P.b_bp = C.b_bp, P.b_gain = C.b_gain;
  P.sp_srcmin = C.sp_srcmin, P.sp_srcmax = C.sp_srcmax, P.sp_kin = C.sp_kin, P.sp_kout = C.sp_kout;
  P.sp_pa = C.sp_pa, P.sp_pb = C.sp_pb, P.sp_qa = C.sp_qa, P.sp_qb = C.sp_qb, P.sp_qc = C.sp_qc;
  P.sp_dmin = C.sp_dmin, P.sp_dmax = C.sp_dmax;
  P.n_peak = C.n_peak, P.n_rein_off = C.n_rein_off, P.n_rein_scale = C.n_rein_scale, P.n_hable_inv = C.n_hable_inv;
  P.n_mob_j = C.n_mob_j, P.n_mob_a = C.n_mob_a, P.n_mob_b = C.n_mob_b, P.n_mob_scale = C.n_mob_scale;
  P.x_peak = C.x_peak, P.x_avg = C.x_avg;
}

// Parameters of the specialised fast kernel (h2s_fast.hip): the same chain
// with every scale folded into constants.
struct FastParams : CurveConsts {
  int W, H, cw, ch;                // luma / chroma geometry (W % 64 == 0)
  int chroma_edge;                 // S1 upsampler edge rule (chroma_edge_at)
  unsigned nbx, nby, nframes;      // 64 x 32 tiles per row / column, frames
  int tpb;                         // tiles walked by one block (k_tile prefetches tile i+1 during tile i)
  const uint8_t* in[3];
  long long in_ls[3], in_fp[3];
  uint8_t* out[3];
  long long out_ls[3], out_fp[3];
  int in_bytes[3], out_bytes[3];   // plane extents for buffer resources (clamped to 2^31-1)
  // S1: R'G'B' = k + ys*Y + a*{U,V}; index [0] even columns (x4), [1] odd (x8)
  float ys, k_r, k_g, k_b;
  float a_rv[2], a_gv[2], a_gu[2], a_bu[2];
  float log2_lin_scale;
  float log2_pq_scale;             // log2(10000 / npl): the PQ EOTF table's scale (the IPT decode reads it for HLG input too)
  float y_off_c, c_mid;            // k_tile staging: Y' = Y*ys + y_off_c, chroma centred on c_mid
  // S2
  float lr, lg, lb, desat;
  float rein_p, rein_k;
  float hable_peak_inv;
  float hable_ka, hable_kb;        // 0.14 / hable(peak), (1/60) / hable(peak): hable(x)/x = (0.14 x + 1/60) / D(x)
  float mob_j, mob_a, mob_b, mob_k;
  float npl_1e4, e4_npl;
  float tw_fold;                   // BT.2390 / spline on PQ input: npl / target white (the EOTF table is npl-scaled)
  float b_e1min;                   // PQ code of sig = 1e-6 (BT.2390 / spline e1 lower bound)
  // libplacebo branch (k_tile<..., LP = 1>): 255 (x ainv)^(1/2.4) - 255 b =
  // exp2(log2(x)/2.4 + lp_k1) - lp_k2, x clamped to [0, lp_xmax] (v >= 1 above);
  // lut3d's 8-bit coordinate (q * inv255) * nm1; BT.709 rows at depth q
  float lp_k1, lp_k2, lp_xmax, nm1, inv255, qscale, c56;
  float k709[3], kcb[3], kcr[3];
  // lp_tone = IPT: RGB (npl units) -> LMS / 10000 (npl/10000 folded in); LMS
  // -> RGB; the PQ encode as PQI_NSEG cubic segments (pqi)
  int lp_ipt;
  // rgba8 download (the LP instances): code = floor(e lp_qs_f + qoff), e the
  // 255-scaled encode, qoff = lp_qo + (lp_dith ? bayer16 : 0.5) per pixel;
  // in_mask2: the input code mask on a packed pair of samples
  float lp_qs_f, lp_qo;
  int lp_dith;
  unsigned in_mask2;
  // the Y'CbCr rows applied to lut3d's 8-bit output codes directly (tile
  // kernel, round 6): o = (sum lp_ky[c] code_c + lp_cy, sum lp_kcb[c] code_c,
  // sum lp_kcr[c] code_c), i.e. k709 / kcb / kcr x inv255 x (219 qscale | 56
  // qscale) folded on the host; lp_cy = 16 qscale + 0.5
  float lp_ky[3], lp_kcb[3], lp_kcr[3], lp_cy;
  float ipt_r2l[9], ipt_l2r[9];
  const float4* pqi_tab;
  // libplacebo branch with the LUT off (k_tile<..., LP = 1>): libplacebo's own
  // BT.2020 -> BT.709 conversion (linear matrix, clip) and the nv12 download
  int lut_off;
  float m709[9];
  float n_nw, tw_1e4;              // npl / target white (npl units -> NORM); target white / 10000
  const CurveConsts* cv_frames;    // dynamic peak: one curve per frame of the launch (else null:
                                   // the base CurveConsts is the batch's curve)
  // S3/S4: lattice coordinates and byte offsets (float4 records)
  float log2_nm1, s_max, stride_g, stride_b;  // byte strides 12N, 12N^2 (as floats)
  float x_max;                                 // largest x with (N-1) x^(1/2.4) < N-1 (margin)
  int og, ob, cr, cg, cb, c111;                // corner byte offsets
  const float* lut_yuv;                        // 12-byte records (Y', Cb', Cr')
  int lut_bytes;
  const unsigned* lut8x;                       // libplacebo branch: lut3d's 8-bit output per rgba code triple
                                               // (bit-interleaved index; R | G << 8 | B << 16), k_build_lut8x
  // S6..S8
  const uint16_t* eq_lut;
  int eq_n;
  float c_bias;
  int shift_out, out8;
  int rep_rs;                      // S8: 8 - shift_out (bit replication) or 31 (shift)
  int dither;                      // S6 ordered dither at the 8-bit quantiser
  // BICUBIC chroma (two-pass, one frame per launch): per-pixel (Cb, Cr) into
  // chr444 (row pitch chr_w) instead of the 2x2 sums; inv_c56 = 1 / (56 q)
  float2* chr444;
  int chr_w;
  float inv_c56;
  // k_tile's branch-free tiles: every staged luma <= safe_y and every centred
  // chroma code <= safe_c bound E below the EOTF table's end (resolve_fast)
  float safe_y, safe_c;
  // S1 PQ EOTF (x 10000/npl) as a piecewise cubic: segment i covers
  // E in [i, i+1)/PQ_SEG, coefficients (c3, c2, c1, c0) of t = E*PQ_SEG - i
  const float4* pq_tab;
  // debug instances (k_tile<..., DBG>): stage planes of frame 0, row pitch
  // dbg_w floats; the float4 RGB lattice for stage 4; 1 / (N-1)
  float* dbg;
  int dbg_w;
  const float4* dbg_lut;
  float inv_nm1;
};

constexpr int TBW = 64, TBH = 32;   // k_tile: luma tile of one block
constexpr int PQ_SEG = 128;          // segments per unit of E
constexpr int PQ_NSEG = 240;         // table covers E in [0, 1.875)
constexpr float PQ_EMAX = 1.875f;    // above: exact transcendental path
constexpr int PQI_OCT0 = -64;        // PQ encode table: first octave 2^-64 (x 10000 nits)
constexpr int PQI_PER_OCT = 8;       // segments per octave (exponent + top 3 mantissa bits)
constexpr int PQI_NSEG = 78 * PQI_PER_OCT;   // octaves 2^-64 .. 2^14
// the table holds PQI_NSEG + 1 entries: [0] = PQ(0) as a constant (y <= 0,
// and y below the first octave), [1 + s] = segment s
constexpr int PQI_NTAB = PQI_NSEG + 1;

struct YuvLutConsts {
  float s, k709[3], kcb[3], kcr[3];
  int rgb;  // 1: plain R'G'B' records (the libplacebo branch truncates lut3d's output before Y'CbCr)
};

// ---- fast transcendentals (v_log_f32 / v_exp_f32 / v_rcp_f32) ----------
__device__ __forceinline__ float flog2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// x^p for x >= 0 (x == 0 -> 0 for p > 0)
__device__ __forceinline__ float fpow(float x, float p) { return fexp2(p * flog2(x)); }
// the generic chain's pow and exp: the oracle's own, glibc 2.35 powf / expf
// (the x86-64 FMA build: double-precision table + polynomial forms, one
// rounding to float), over the tables scripts/gen_libm_tables.py reads out of
// the libm the oracle links (h2s_libm.h; tests/test_libm_tables.py pins them).
// Their last rounding is not the correctly rounded one for a few inputs in
// 10^4, and the PQ EOTF amplifies a pow ulp ~500-fold (m2 = 78.84; the
// xp - c1 and c2 - c3 xp cancellations): enough to flip the libplacebo
// branch's 8-bit rgba rounding.  The generic kernel is the branch's exact
// path (H2S_OPT_LP_EXACT; h2s_kernels.hip is built without FMA contraction, in
// the oracle's operation order); the tile kernel keeps its own fast forms.
// (no FMA contraction inside: the forms round where glibc's do, whichever
// translation unit includes them; tests/test_libm_tables.py checks the device
// forms bit for bit against the libm through h2stest_libm)
__device__ __forceinline__ float libm_exp2_tail(double xd, double shift, const double* C) {
#pragma clang fp contract(off)
  double kd = xd + shift;
  const unsigned long long ki = (unsigned long long)__double_as_longlong(kd);
  kd -= shift;
  const double r = xd - kd;
  const unsigned long long t = libm::EXP2F_TAB[ki & 31] + (ki << 47);
  const double s = __longlong_as_double((long long)t);
  const double z = __builtin_fma(C[0], r, C[1]);
  const double r2 = r * r;
  double y = __builtin_fma(C[2], r, 1.0);
  y = __builtin_fma(z, r2, y);
  return (float)(y * s);
}
// powf for x >= 0 (the chain's uses); other bases take the double form
__device__ __forceinline__ float libm_powf(float x, float yf) {
#pragma clang fp contract(off)
  if (!(x > 0.0f) || !(x < __builtin_inff()) || yf == 0.0f || !(fabsf(yf) < __builtin_inff()))
    return (float)pow((double)x, (double)yf);
  unsigned ix = __float_as_uint(x);
  if (ix < 0x00800000u) ix = __float_as_uint(x * 0x1p23f) - (23u << 23);  // subnormal
  const unsigned tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) & 15u);
  const unsigned top = tmp & 0xff800000u;
  const unsigned iz = ix - top;
  const int k = (int)top >> 23;
  const double invc = libm::POWF_LOG2_TAB[i][0], logc = libm::POWF_LOG2_TAB[i][1];
  const double z = (double)__uint_as_float(iz);
  const double* A = libm::POWF_LOG2_POLY;
  const double r = __builtin_fma(z, invc, -1.0);
  const double y0 = logc + (double)k;
  const double r2 = r * r;
  double y = __builtin_fma(A[0], r, A[1]);
  const double p = __builtin_fma(A[2], r, A[3]);
  const double r4 = r2 * r2;
  double q = __builtin_fma(A[4], r, y0);
  q = __builtin_fma(p, r2, q);
  y = __builtin_fma(y, r4, q);
  const double ylogx = (double)yf * y;
  if ((((unsigned long long)__double_as_longlong(ylogx) >> 47) & 0xffffu) >= (0x405f800000000000ull >> 47)) {
    if (ylogx > 0x1.fffffffd1d571p+6) return __builtin_inff();
    if (ylogx <= -150.0) return 0.0f;
  }
  return libm_exp2_tail(ylogx, libm::EXP2F_SHIFT_SCALED, libm::EXP2F_POLY);
}
__device__ __forceinline__ float libm_expf(float x) {
  if (x != x) return x;
  if (x > 0x1.62e42ep6f) return __builtin_inff();
  if (x < -0x1.9fe368p6f) return 0.0f;
  return libm_exp2_tail(libm::EXP2F_INVLN2_SCALED * (double)x, libm::EXP2F_SHIFT, libm::EXP2F_POLY_SCALED);
}
__device__ __forceinline__ float apow(float x, float p) { return libm_powf(x, p); }
__device__ __forceinline__ float aexp(float x) { return libm_expf(x); }
__device__ __forceinline__ float clamp01(float x) { return __builtin_amdgcn_fmed3f(x, 0.0f, 1.0f); }

// ST 2084 constants (exact binary values, as zimg defines them)
#define PQ_M1 0.1593017578125f
#define PQ_M2 78.84375f
#define PQ_C1 0.8359375f
#define PQ_C2 18.8515625f
#define PQ_C3 18.6875f
#define HLG_A 0.17883277f
#define HLG_B 0.28466892f
#define HLG_C 0.55991073f

// S1 transfer: zimg st_2084_eotf (normalised, 1.0 = 10000 nits)
__device__ __forceinline__ float pq_eotf(float x) {
  if (!(x > 0.0f)) return 0.0f;
  float xpow = apow(x, 1.0f / PQ_M2);
  float num = fmaxf(xpow - PQ_C1, 0.0f);
  float den = fmaxf(PQ_C2 - PQ_C3 * xpow, 1.17549435e-38f);
  return apow(num / den, 1.0f / PQ_M1);
}

// ST 2084 inverse EOTF (BT.2390 works in the PQ domain)
__device__ __forceinline__ float pq_encode(float y) {
  float ym = apow(fmaxf(y, 0.0f), PQ_M1);
  return apow((PQ_C1 + PQ_C2 * ym) / (1.0f + PQ_C3 * ym), PQ_M2);
}

// zimg arib_b67_inverse_oetf
__device__ __forceinline__ float hlg_inv_oetf(float x) {
  x = fmaxf(x, 0.0f);
  if (x <= 0.5f) return (x * x) * (1.0f / 3.0f);
  return (aexp((x - HLG_C) / HLG_A) + HLG_B) * (1.0f / 12.0f);
}

// vf_tonemap hable()
__device__ __forceinline__ float hable(float in) {
  const float a = 0.15f, b = 0.50f, c = 0.10f, d = 0.20f, e = 0.02f, f = 0.30f;
  return (in * (in * a + b * c) + d * e) / (in * (in * a + b) + d * f) - e / f;
}

// libplacebo spline on a PQ-domain signal: quadratic toe below the knee,
// cubic shoulder above it (constants: spline_consts in h2s_api.hip)
// (the oracle's spline_pq_f expression: unfused where the translation unit
// does not contract, as h2s_kernels.hip)
template <class K>
__device__ __forceinline__ float spline_pq(const K& P, float e) {
  const float x = fminf(fmaxf(e, P.sp_srcmin), P.sp_srcmax) - P.sp_kin;
  const float y = x > 0.0f ? ((P.sp_qa * x + P.sp_qb) * x + P.sp_qc) * x : (P.sp_pa * x + P.sp_pb) * x;
  return fminf(fmaxf(y + P.sp_kout, P.sp_dmin), P.sp_dmax);
}

// libplacebo bt2390 black-point adaptation on the normalised curve output
// (x += minLum (1 - x)^bp, x = gain (x - minLum) + minLum, for x < 1): the
// tile kernel's form (HLG input), bp = 4 as two squarings
__device__ __forceinline__ float bt2390_black(float mn, float bp, float gain, float x) {
  if (!(mn > 0.0f) || !(x < 1.0f)) return x;
  const float om = 1.0f - x;
  const float pw = bp == 4.0f ? (om * om) * (om * om) : powf(om, bp);
  x += mn * pw;
  return gain * (x - mn) + mn;
}

// libplacebo bt2390 on a PQ-domain signal, in the oracle's operation order
// (oracle bt2390_pq: divisions by the range and by 1 - ks, powf for any bp)
__device__ __forceinline__ float bt2390_pq(const KParams& P, float e1) {
  float e1n = (e1 - P.b_srcmin) / P.b_range;
  e1n = fmaxf(fminf(e1n, 1.0f), 0.0f);  // clip to the source range (NaN -> 1)
  const float ks = P.b_ks, ml = P.b_maxlum;
  float e2 = e1n;
  if (ks < 1.0f && e1n > ks) {
    float t = (e1n - ks) / (1.0f - ks);
    float t2 = t * t, t3 = t2 * t;
    e2 = (2.0f * t3 - 3.0f * t2 + 1.0f) * ks + (t3 - 2.0f * t2 + t) * (1.0f - ks) + (-2.0f * t3 + 3.0f * t2) * ml;
  }
  if (P.b_minlum > 0.0f && e2 < 1.0f) {
    const float mn = P.b_minlum;
    e2 += mn * apow(1.0f - e2, P.b_bp);
    e2 = P.b_gain * (e2 - mn) + mn;
  }
  return e2 * P.b_range + P.b_srcmin;
}

// libplacebo branch, h2s_lp_tone IPT (oracle tone_ipt): the PQ-domain curve
// on the intensity of IPT-PQ, P and T kept, i.e. L'M'S' += I' - I.  In double
// around the float curve, as the oracle: the LMS -> RGB rows turn float32
// EOTF noise into large errors on channels they cancel to near zero
__device__ __forceinline__ double pq_encode_dd(double y) {
  const double ym = pow(fmax(y, 0.0), (double)PQ_M1);
  return pow(((double)PQ_C1 + (double)PQ_C2 * ym) / (1.0 + (double)PQ_C3 * ym), (double)PQ_M2);
}
__device__ __forceinline__ double pq_eotf_dd(double e) {
  if (!(e > 0.0)) return 0.0;
  const double xp = pow(e, 1.0 / (double)PQ_M2);
  return pow(fmax(xp - (double)PQ_C1, 0.0) / ((double)PQ_C2 - (double)PQ_C3 * xp), 1.0 / (double)PQ_M1);
}
// libplacebo's reinhard / hable / mobius in NORM units (oracle lp_norm_curve)
__device__ __forceinline__ float lp_norm_curve(const KParams& P, float x) {
  x = fminf(fmaxf(x, 0.0f), P.n_peak);
  if (P.tonemap == 4) return P.n_rein_scale * x / (x + P.n_rein_off);
  if (P.tonemap == 5) return hable(x) / hable(P.n_peak);   // (oracle: hable(x) / hable(pk))
  return x <= P.n_mob_j ? x : P.n_mob_scale * (x + P.n_mob_a) / (x + P.n_mob_b);
}

__device__ __forceinline__ void tone_ipt(const KParams& P, float& r, float& g, float& b) {
  const double s = P.ipt_npl;
  const double v0 = fmin((double)r, 1e6) * s, v1 = fmin((double)g, 1e6) * s, v2 = fmin((double)b, 1e6) * s;
  double q[3];
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = pq_encode_dd(P.ipt_r2l[3 * k] * v0 + P.ipt_r2l[3 * k + 1] * v1 + P.ipt_r2l[3 * k + 2] * v2);
  const double I = 0.4 * q[0] + 0.4 * q[1] + 0.2 * q[2];
  double I2;
  if (P.tonemap == 8) I2 = spline_pq(P, (float)I);
  else if (P.tonemap == 7) I2 = bt2390_pq(P, (float)I);
  else I2 = pq_encode_dd((double)lp_norm_curve(P, (float)(pq_eotf_dd(I) * P.ipt_os)) * P.ipt_tw);
  const double dI = I2 - I;
  double l[3];
#pragma unroll
  for (int k = 0; k < 3; k++) l[k] = pq_eotf_dd(q[k] + dI);
  const double os = P.ipt_os;
  r = (float)((P.ipt_l2r[0] * l[0] + P.ipt_l2r[1] * l[1] + P.ipt_l2r[2] * l[2]) * os);
  g = (float)((P.ipt_l2r[3] * l[0] + P.ipt_l2r[4] * l[1] + P.ipt_l2r[5] * l[2]) * os);
  b = (float)((P.ipt_l2r[6] * l[0] + P.ipt_l2r[7] * l[1] + P.ipt_l2r[8] * l[2]) * os);
}

// S2: vf_tonemap tonemap() on one linear RGB pixel (units of npl)
__device__ __forceinline__ void tonemap_px(const KParams& P, float& r, float& g, float& b) {
  float sig, sig_orig;
  if (P.lp_ipt) {   // set on the libplacebo branch only
    tone_ipt(P, r, g, b);
    return;
  }
  if (P.lp_norm) {  // libplacebo branch, max(R,G,B) gain (oracle tonemap_px)
    r = fminf(r, 1e6f), g = fminf(g, 1e6f), b = fminf(b, 1e6f);
    sig = fmaxf(fmaxf(fmaxf(r, g), b), 1e-6f);
    const float k = lp_norm_curve(P, sig * P.n_nw) / sig;
    r *= k, g *= k, b *= k;
    return;
  }
  if (P.tonemap == 8 /* SPLINE */) {
    sig = fmaxf(fmaxf(fmaxf(r, g), b), 1e-6f);
    const float s2 = pq_eotf(spline_pq(P, pq_encode(sig * P.npl_1e4))) * P.e4_npl;
    const float k = s2 / sig;
    r *= k, g *= k, b *= k;
    return;
  }
  if (P.tonemap == 7 /* BT2390 */) {
    sig = fmaxf(fmaxf(fmaxf(r, g), b), 1e-6f);
    float s2 = pq_eotf(bt2390_pq(P, pq_encode(sig * P.npl_1e4))) * P.e4_npl;
    float k = s2 / sig;
    r *= k, g *= k, b *= k;
    return;
  }
  if (P.desat_on) {
    float luma = P.lr * r + P.lg * g + P.lb * b;
    float ob = fmaxf(luma - P.desat, 1e-6f) / fmaxf(luma, 1e-6f);
    r = r * (1.0f - ob) + luma * ob;
    g = g * (1.0f - ob) + luma * ob;
    b = b * (1.0f - ob) + luma * ob;
  }
  sig = fmaxf(fmaxf(fmaxf(r, g), b), 1e-6f);
  sig_orig = sig;
  switch (P.tonemap) {
    case 1:  // LINEAR
      sig = sig * P.lin_k;
      break;
    case 2:  // GAMMA
      sig = sig > 0.05f ? apow(sig * P.gam_inv_peak, P.gam_inv_param) : sig * P.gam_low_k;
      break;
    case 3:  // CLIP
      sig = clamp01(sig * P.clip_k);
      break;
    case 4:  // REINHARD
      sig = sig / (sig + P.rein_p) * P.rein_k;
      break;
    case 5:  // HABLE
      sig = hable(sig) * P.hable_peak_inv;
      break;
    case 6:  // MOBIUS
      sig = sig <= P.mob_j ? sig : P.mob_k * (sig + P.mob_a) / (sig + P.mob_b);
      break;
    default:
      break;
  }
  float k = sig / sig_orig;
  r *= k, g *= k, b *= k;
}

// S3: zimg rec_1886_inverse_eotf
__device__ __forceinline__ float bt1886_inv(float x) {
  return x > 0.0f ? apow(x, 1.0f / 2.4f) : 0.0f;
}

// S4: vf_lut3d sanitizef + clip + interp_tetrahedral.  The lattice is in
// .cube order (red fastest): index(r,g,b) = r + g*N + b*N^2.  Case selection
// uses the same strict comparisons as interp_tetrahedral, expressed as
// selects instead of branches (no divergence); the weights and the term order
// are the reference's.
__device__ __forceinline__ float lut_coord(float x, float lut_max) {
  x = (x == x) ? x : 0.0f;  // NaN -> 0 (sanitizef); +-inf clip below
  return __builtin_amdgcn_fmed3f(x * lut_max, 0.0f, lut_max);
}

// tetrahedral blend at lattice coordinates s in [0, N-1] (lut3d interp_tetrahedral)
__device__ __forceinline__ void lut3d_tetra_at(const KParams& P, float sr, float sg, float sb, float& r, float& g,
                                               float& b) {
  const int pr = (int)sr, pg = (int)sg, pb = (int)sb;
  const int last = P.lut_n - 1;
  const int str = pr < last ? 1 : 0;
  const int stg = pg < last ? P.lut_sg : 0;
  const int stb = pb < last ? P.lut_sb : 0;
  const float dr = sr - (float)pr, dg = sg - (float)pg, db = sb - (float)pb;
  const bool rg = dr > dg, gb = dg > db, rb = dr > db, bg = db > dg, br = db > dr;
  float x1, x2, x3;
  int o1, o2;
  if (rg) {
    if (gb) { x1 = dr; x2 = dg; x3 = db; o1 = str; o2 = stg; }
    else if (rb) { x1 = dr; x2 = db; x3 = dg; o1 = str; o2 = stb; }
    else { x1 = db; x2 = dr; x3 = dg; o1 = stb; o2 = str; }
  } else {
    if (bg) { x1 = db; x2 = dg; x3 = dr; o1 = stb; o2 = stg; }
    else if (br) { x1 = dg; x2 = db; x3 = dr; o1 = stg; o2 = stb; }
    else { x1 = dg; x2 = dr; x3 = db; o1 = stg; o2 = str; }
  }
  const int base = pr + pg * P.lut_sg + pb * P.lut_sb;
  const float4 c000 = P.lut[base];
  const float4 c1 = P.lut[base + o1];
  const float4 c2 = P.lut[base + o1 + o2];
  const float4 c111 = P.lut[base + str + stg + stb];
  const float w0 = 1.0f - x1, w1 = x1 - x2, w2 = x2 - x3, w3 = x3;
  r = w0 * c000.x + w1 * c1.x + w2 * c2.x + w3 * c111.x;
  g = w0 * c000.y + w1 * c1.y + w2 * c2.y + w3 * c111.y;
  b = w0 * c000.z + w1 * c1.z + w2 * c2.z + w3 * c111.z;
}

__device__ __forceinline__ void lut3d_tetra(const KParams& P, float& r, float& g, float& b) {
  lut3d_tetra_at(P, lut_coord(r, P.lut_max), lut_coord(g, P.lut_max), lut_coord(b, P.lut_max), r, g, b);
}

// libplacebo branch: BT.1886 encode against the target black (oracle lp_encode)
__device__ __forceinline__ float lp_encode(const KParams& P, float x) {
  x = x > 0.0f ? x : 0.0f;
  return apow(x / P.enc_a, 1.0f / 2.4f) - P.enc_b;
}

// libplacebo branch: rgba8 download (round to nearest), then vf_lut3d's 8-bit
// path: coordinate clip((q / 255) (N-1)), tetrahedral, output truncated to
// 8 bits; returns the 8-bit values / 255
// qoff: lp_qoff (the range=tv offset and the rounding / dither offset)
__device__ __forceinline__ float rgba8_q(const KParams& P, float v, float qoff) {
  return floorf(clamp01(v) * P.lp_qs + qoff);   // (two roundings, as the oracle's rgba8_q)
}

// 16 x 16 Bayer matrix (M_2n = 4 M_n + M_1 per 2 x 2 block, M_1 = [0 2; 3 1])
// as a dither offset (M + 0.5) / 256 in (0, 1): the h2s_lp_dither ORDERED model
__host__ __device__ __forceinline__ float bayer16(int x, int y) {
  int m = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int bx = (x >> i) & 1, by = (y >> i) & 1;
    m += (2 * (bx ^ by) + by) << (2 * (3 - i));
  }
  return ((float)m + 0.5f) * (1.0f / 256.0f);
}

// the rgba8 download's offset for pixel (x, y)
__device__ __forceinline__ float lp_qoff(const KParams& P, int x, int y) {
  return P.lp_qo + (P.lp_dith ? bayer16(x, y) : 0.5f);
}

__device__ __forceinline__ void lut3d_8bit(const KParams& P, float& r, float& g, float& b, float qoff) {
  const float sf = 1.0f / 255.0f;
  // lut3d_tetra multiplies by lut_max and clips; (q * 1/255) is its input
  r = rgba8_q(P, r, qoff) * sf, g = rgba8_q(P, g, qoff) * sf, b = rgba8_q(P, b, qoff) * sf;
  lut3d_tetra(P, r, g, b);
  const float R = fminf(fmaxf(truncf(r * 255.0f), 0.0f), 255.0f);
  const float G = fminf(fmaxf(truncf(g * 255.0f), 0.0f), 255.0f);
  const float B = fminf(fmaxf(truncf(b * 255.0f), 0.0f), 255.0f);
  r = R * sf, g = G * sf, b = B * sf;
}

// S3 -> S4 as 16-bit R'G'B' (h2s_lut_input RGB48; oracle rgb48_q /
// lut3d_16bit): round to 16 bits, lut3d's 16-bit coordinate, output truncated
__device__ __forceinline__ float rgb48_q(float v) { return floorf(clamp01(v) * 65535.0f + 0.5f); }
__device__ __forceinline__ void lut3d_16bit(const KParams& P, float& r, float& g, float& b) {
  const float scale = (1.0f / 65535.0f) * P.lut_max;
  const float sr = __builtin_amdgcn_fmed3f(rgb48_q(r) * scale, 0.0f, P.lut_max);
  const float sg = __builtin_amdgcn_fmed3f(rgb48_q(g) * scale, 0.0f, P.lut_max);
  const float sb = __builtin_amdgcn_fmed3f(rgb48_q(b) * scale, 0.0f, P.lut_max);
  float orr, og, ob;
  lut3d_tetra_at(P, sr, sg, sb, orr, og, ob);
  r = fminf(fmaxf(truncf(orr * 65535.0f), 0.0f), 65535.0f) / 65535.0f;
  g = fminf(fmaxf(truncf(og * 65535.0f), 0.0f), 65535.0f) / 65535.0f;
  b = fminf(fmaxf(truncf(ob * 65535.0f), 0.0f), 65535.0f) / 65535.0f;
}

// S1 (after upsampling) .. S4 on one pixel.  UPTO = last stage to apply.
template <int UPTO>
__device__ __forceinline__ void chain_px(const KParams& P, float y, float cb, float cr, float& r, float& g,
                                         float& b, float qoff = 0.5f) {
  float er = y + P.m_rcr * cr;
  float eg = y + P.m_gcb * cb + P.m_gcr * cr;
  float eb = y + P.m_bcb * cb;
  if (P.transfer == 1) {  // HLG: inverse OETF + OOTF (gamma 1.2 at 1000 nits)
    r = hlg_inv_oetf(er), g = hlg_inv_oetf(eg), b = hlg_inv_oetf(eb);
    float ys = 0.2627f * r + 0.6780f * g + 0.0593f * b;
    float w = ys > 0.0f ? P.lin_scale * apow(ys, 0.2f) : 0.0f;
    r *= w, g *= w, b *= w;
  } else {
    r = pq_eotf(er) * P.lin_scale;
    g = pq_eotf(eg) * P.lin_scale;
    b = pq_eotf(eb) * P.lin_scale;
  }
  if (UPTO == 1) return;
  tonemap_px(P, r, g, b);
  if (UPTO == 2) return;
  if (P.pipe == PIPE_LIBPLACEBO) {
    if (P.lut_enabled) {
      r = lp_encode(P, r), g = lp_encode(P, g), b = lp_encode(P, b);
      if (UPTO == 3) return;
      lut3d_8bit(P, r, g, b, qoff);
    } else {
      float mr = P.m709[0] * r + P.m709[1] * g + P.m709[2] * b;
      float mg = P.m709[3] * r + P.m709[4] * g + P.m709[5] * b;
      float mb = P.m709[6] * r + P.m709[7] * g + P.m709[8] * b;
      r = clamp01(lp_encode(P, mr)), g = clamp01(lp_encode(P, mg)), b = clamp01(lp_encode(P, mb));
    }
    return;
  }
  if (P.lut_enabled) {
    r = bt1886_inv(r), g = bt1886_inv(g), b = bt1886_inv(b);
    if (UPTO == 3) return;
    if (P.lut_in16) {
      lut3d_16bit(P, r, g, b);
      return;
    }
    lut3d_tetra(P, r, g, b);
  } else {
    float mr = P.m709[0] * r + P.m709[1] * g + P.m709[2] * b;
    float mg = P.m709[3] * r + P.m709[4] * g + P.m709[5] * b;
    float mb = P.m709[6] * r + P.m709[7] * g + P.m709[8] * b;
    r = clamp01(bt1886_inv(mr)), g = clamp01(bt1886_inv(mg)), b = clamp01(bt1886_inv(mb));
  }
}

__device__ __forceinline__ int quant(float v, int qmax) {
  int i = (int)floorf(v + 0.5f);
  return min(max(i, 0), qmax);
}

// swscale ff_dither_8x8_128 (1/128 LSB): the H2S_DITHER_ORDERED rounding
__device__ __forceinline__ float dither_off(int x, int y) {
  constexpr unsigned char T[8][8] = {
      {36, 68, 60, 92, 34, 66, 58, 90},   {100, 4, 124, 28, 98, 2, 122, 26},
      {52, 84, 44, 76, 50, 82, 42, 74},   {116, 20, 108, 12, 114, 18, 106, 10},
      {32, 64, 56, 88, 38, 70, 62, 94},   {96, 0, 120, 24, 102, 6, 126, 30},
      {48, 80, 40, 72, 54, 86, 46, 78},   {112, 16, 104, 8, 118, 22, 110, 14}};
  return (float)T[y & 7][x & 7] * (1.0f / 128.0f);
}

__device__ __forceinline__ int quant_o(float v, float off, int qmax) {
  int i = (int)floorf(v + off);
  return min(max(i, 0), qmax);
}

// S8 expansion of a quantised code to the output depth
__device__ __forceinline__ int expand_code(const KParams& P, int v) {
  if (!P.shift_out) return v;
  return P.expand_rep ? (v << P.shift_out) | (v >> (8 - P.shift_out)) : v << P.shift_out;
}

}  // namespace h2s
