// h2s_peak.h — the per-frame tone curve under dynamic peak detection
// (libplacebo peak_detect=1, src/utils.py:445-449; PARITY UNPINNED: the model
// is DESIGN.md §4.6), as host/device code: the percentile of a frame's
// PQ(max R,G,B) histogram, the IIR over frames with the scene-change bypass,
// and the BT.2390 / spline / libplacebo-NORM curve constants of the smoothed
// peak in the tile kernel's folded form (CurveConsts).
//
// One definition serves the host (the static curve of h2s_set_params) and the
// device (k_peak_stats* + k_peak_finish in h2s_kernels.hip: h2s_process with
// peak_detect queues the statistics, then the per-frame fold with the IIR and
// curve records in its last block, then the conversion, on its stream with no
// host round trip; k_peak_curves serves h2s_peak_feed), so the two cannot
// drift apart.  The oracle's statement is
// oracle/h2s_oracle.c (PeakState, resolve).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "h2s_device.h"

namespace h2s {

constexpr int PEAK_BLOCKS = 128;      // partial (max, sum) records per frame (k_peak_stats*), default (round 6: 64 -> 128)
constexpr int PEAK_BLOCKS_MAX = 256;  // ... at most (H2S_OPT_TEST_PEAK_BLOCKS A/B; one per finish thread)
constexpr int PEAK_BINS = 1024;  // percentile histogram bins over PQ [0, 1]

// the PQ levels of the SDR target that every curve set-up needs: PQ(0), PQ of
// the target white and black (nits / 10000), pq_refs below.  Host-made once
// per launch for the device's per-frame records, so that k_peak_finish's
// serial tail spends its double-precision powers on the frame's peak only
struct PqRefs {
  double smin, white, black;
};

// the launch-constant inputs of a frame's curve (resolved h2s_params)
struct PeakModel {
  double t_white, t_black;            // SDR target, nits
  double knee_off, contrast, tm_param;
  double static_peak;                 // the clamp's top: the metadata / default peak (units of 100 nits)
  double smoothing, scene_low, scene_high, percentile, min_peak;  // vf_libplacebo options (min_peak x 100 nits)
  double iir_a;                       // the IIR coefficient 1 - exp(-1 / smoothing) (1: no smoothing), host-made
  double npx;                         // pixels per frame
  int nblocks;                        // partial records per frame
  int pct;                            // percentile < 100: histograms present
  int family;                         // the curve the records serve: 7 BT.2390, 8 spline, else libplacebo NORM
  PqRefs pq;                          // pq_refs(t_white, t_black), host-made
};

// the smoothing state carried from frame to frame and call to call
// (h2s_peak_state reads it back)
struct PeakState {
  double max, avg, peak;
  long long frames;
};

// The buffers of a statistics launch (k_peak_stats* then k_peak_finish, in
// h2s_kernels.hip).  The histograms and the counter are zero on entry and are
// left zero (h2s_api.hip clears them once, at allocation).
struct PeakTail {
  PeakModel M;
  double2* fstat;      // nframes: the frames' (measurement, average)
  unsigned* hist;      // nframes x PEAK_BINS (M.pct)
  unsigned* done;      // one counter (frames folded)
  PeakState* st;       // null: the statistics only (h2s_peak_stats)
  CurveConsts* out;    // nframes curve records, or null
  int nframes;
  int form;            // PQ statistics form: 0 = 32-pixel quad units (default), 1 = 8-pixel row chunks (test hook A/B)
};

__host__ __device__ inline double hd_pq_encode(double y) {
  const double m1 = 0.1593017578125, m2 = 78.84375, c1 = 0.8359375, c2 = 18.8515625, c3 = 18.6875;
  const double ym = pow(fmax(y, 0.0), m1);
  return pow((c1 + c2 * ym) / (1.0 + c3 * ym), m2);
}

// ST 2084 EOTF in double (normalised: 1.0 = 10000 nits)
__host__ __device__ inline double hd_pq_eotf(double e) {
  const double m1 = 2610.0 / 16384.0, m2 = 2523.0 / 4096.0 * 128.0, c1 = 3424.0 / 4096.0, c2 = 2413.0 / 4096.0 * 32.0,
               c3 = 2392.0 / 4096.0 * 32.0;
  if (!(e > 0.0)) return 0.0;
  const double xp = pow(e, 1.0 / m2);
  const double num = xp - c1 > 0.0 ? xp - c1 : 0.0;
  return pow(num / (c2 - c3 * xp), 1.0 / m1);
}

__host__ __device__ inline PqRefs pq_refs(double t_white, double t_black) {
  return PqRefs{hd_pq_encode(0.0), hd_pq_encode(t_white / 10000.0), hd_pq_encode(t_black / 10000.0)};
}

__host__ __device__ inline float hd_hable(float in) {
  const float a = 0.15f, b = 0.50f, c = 0.10f, d = 0.20f, e = 0.02f, f = 0.30f;
  return (in * (in * a + b * c) + d * e) / (in * (in * a + b) + d * f) - e / f;
}

// libplacebo's reinhard / hable / mobius in NORM units (1 = target white) for
// a source peak (units of 100 nits); oracle lp_norm_curve.  K: KParams or
// CurveConsts (same field names)
template <class K>
__host__ __device__ inline void lp_norm_consts(double peak, double tm_param, double t_white, K* k) {
  const float pk = (float)(peak * 100.0 / t_white);
  k->n_peak = pk;
  const float ct = isnan(tm_param) ? 0.5f : (float)tm_param;
  k->n_rein_off = (1.0f - ct) / ct;
  k->n_rein_scale = (pk + k->n_rein_off) / pk;
  k->n_hable_inv = 1.0f / hd_hable(pk);
  const float j = isnan(tm_param) ? 0.3f : (float)tm_param;
  const float a = -j * j * (pk - 1.0f) / (j * j - 2.0f * j + pk);
  const float b = (j * j - 2.0f * j * pk + pk) / fmaxf(1e-6f, pk - 1.0f);
  k->n_mob_j = j, k->n_mob_a = a, k->n_mob_b = b;
  k->n_mob_scale = (b * b + 2.0f * b * j + j * j) / (b - a);
}

// BT.2390 EETF constants (libplacebo tone_mapping.c bt2390) for a source
// peak (units of 100 nits) and the SDR target [t_black, t_white] nits:
// knee ks = (1 + offset) maxLum - offset, black-point adaptation exponent
// bp = min(1 / minLum, 4) and gain 1 / (1 + minLum / maxLum (1 - maxLum)^bp)
template <class K>
__host__ __device__ inline void bt2390_consts(double peak, double t_white, double t_black, double knee_off, K* k,
                                              const PqRefs& r) {
  const double smin = r.smin, smax = hd_pq_encode(peak * 100.0 / 10000.0);
  const double ml = (r.white - smin) / (smax - smin);
  const double mn = t_black > 0.0 ? (r.black - smin) / (smax - smin) : 0.0;
  const double ks = (1.0 + knee_off) * ml - knee_off;
  const double bp = mn > 0.0 ? fmin(1.0 / mn, 4.0) : 4.0;
  k->b_srcmin = (float)smin;
  k->b_range = (float)(smax - smin);
  k->b_inv_range = (float)(1.0 / (smax - smin));
  k->b_ks = (float)ks;
  k->b_inv_1mks = (float)(1.0 / (1.0 - ks));
  k->b_maxlum = (float)ml;
  k->b_minlum = (float)mn;
  k->b_bp = (float)bp;
  k->b_gain = (float)(ml < 1.0 ? 1.0 / (1.0 + mn / ml * pow(1.0 - ml, bp)) : 1.0);
}

// libplacebo's "spline" tone curve (tone_mapping.c, scaling PL_HDR_PQ;
// PARITY UNPINNED: libplacebo is absent): a single-pivot
// curve in the PQ domain, a quadratic toe below the knee and a cubic
// shoulder above it with zero curvature at the source peak.  The knee
// follows pick_knee with libplacebo's default constants (knee adaptation
// 0.4, minimum 0.1, maximum 0.8, default 0.4; slope tuning 1.5, slope offset
// 0.2).  avg_pq: the frame's average PQ level (peak detection), 0 = unknown.
template <class K>
__host__ __device__ inline void spline_consts(double peak, double avg_pq, double contrast, double t_white,
                                              double t_black, K* k, const PqRefs& r) {
  const double kad = 0.4, kmin = 0.1, kmax = 0.8, kdef = 0.4, st = 1.5, so = 0.2;
  auto mix = [](double a, double b, double t) { return a + (b - a) * t; };
  auto smooth = [](double e0, double e1, double x) {
    double t = (x - e0) / (e1 - e0);
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    return t * t * (3.0 - 2.0 * t);
  };
  (void)t_white, (void)t_black;
  const double smin = r.smin, smax = hd_pq_encode(peak * 100.0 / 10000.0);
  const double dmin = r.black, dmax = r.white;
  double sk = avg_pq > 0.0 ? avg_pq : mix(smin, smax, kdef);
  sk = fmin(fmax(sk, mix(smin, smax, kmin)), mix(smin, smax, kmax));
  const double target = (sk - smin) / (smax - smin);
  const double adapted = mix(dmin, dmax, target);
  const double tuning = 1.0 - smooth(kmax, kdef, target) * smooth(kmin, kdef, target);
  double dk = mix(sk, adapted, mix(kad, 1.0, tuning));
  dk = fmin(fmax(dk, dmin), dmax);
  double ratio = st * (smax / dmax - 1.0);
  ratio = fmin(fmax(ratio, so), 1.0 + so);
  const double slope = pow(hd_pq_eotf(dk) / hd_pq_eotf(sk), (1.0 - contrast) * ratio);
  const double in_min = smin - sk, in_max = smax - sk, out_min = dmin - dk, out_max = dmax - dk;
  const double tq = 2.0 * in_max * in_max;
  k->sp_srcmin = (float)smin, k->sp_srcmax = (float)smax;
  k->sp_kin = (float)sk, k->sp_kout = (float)dk;
  k->sp_pa = (float)((out_min - slope * in_min) / (in_min * in_min));
  k->sp_pb = (float)slope;
  k->sp_qa = (float)((slope * in_max - out_max) / (in_max * tq));
  k->sp_qb = (float)(-3.0 * (slope * in_max - out_max) / tq);
  k->sp_qc = (float)slope;
  k->sp_dmin = (float)dmin, k->sp_dmax = (float)dmax;
}

// BT.2390 / spline constants in the fast kernel's folded form (per launch, or
// per frame under dynamic peak detection).  K holds the plain constants
// (KParams, or a CurveConsts the three *_consts above filled)
template <class K>
__host__ __device__ inline void curve_fast(const K& k, CurveConsts* cc) {
  cc->b_srcmin = k.b_srcmin, cc->b_range = k.b_range, cc->b_inv_range = k.b_inv_range;
  cc->b_ks = k.b_ks, cc->b_inv_1mks = k.b_inv_1mks, cc->b_maxlum = k.b_maxlum;
  cc->b_minlum = k.b_minlum, cc->b_bp = k.b_bp, cc->b_gain = k.b_gain;
  cc->sp_srcmin = k.sp_srcmin, cc->sp_srcmax = k.sp_srcmax, cc->sp_kin = k.sp_kin, cc->sp_kout = k.sp_kout;
  cc->sp_pa = k.sp_pa, cc->sp_pb = k.sp_pb, cc->sp_qa = k.sp_qa, cc->sp_qb = k.sp_qb, cc->sp_qc = k.sp_qc;
  cc->sp_dmin = k.sp_dmin, cc->sp_dmax = k.sp_dmax;
  {
    const double seg = PQ_SEG, smin = k.b_srcmin, range = k.b_range, ks = k.b_ks, ml = k.b_maxlum;
    const double R = range * seg, C = smin * seg + 1.0;
    // (2t^3-3t^2+1) ks + (t^3-2t^2+t)(1-ks) + (-2t^3+3t^2) ml as a3 t^3 + a2 t^2 + a1 t + a0
    const double a3 = ks + 1.0 - 2.0 * ml, a2 = -ks - 2.0 + 3.0 * ml, a1 = 1.0 - ks, a0 = ks;
    cc->b_e1a = k.b_inv_range, cc->b_e1b = (float)(-smin * (double)k.b_inv_range);
    cc->b_ta = k.b_inv_1mks, cc->b_tb = (float)(-ks * (double)k.b_inv_1mks);
    cc->b_c3 = (float)(R * a3), cc->b_c2 = (float)(R * a2), cc->b_c1 = (float)(R * a1), cc->b_c0 = (float)(R * a0 + C);
    cc->b_lr = (float)R, cc->b_lc = (float)C;
    cc->b_thr = ks < 1.0 ? (float)ks : 2.0f;   // ks >= 1: the knee is never reached
    cc->sp_qa_u = (float)(seg * k.sp_qa), cc->sp_qb_u = (float)(seg * k.sp_qb), cc->sp_qc_u = (float)(seg * k.sp_qc);
    cc->sp_pa_u = (float)(seg * k.sp_pa), cc->sp_pb_u = (float)(seg * k.sp_pb);
    cc->sp_k_u = (float)(seg * k.sp_kout + 1.0);
    cc->sp_umin = (float)(seg * k.sp_dmin + 1.0), cc->sp_umax = (float)(seg * k.sp_dmax + 1.0);
    // black-point adaptation in u: 1 - e2 = (R + C - u) / R; u' = gain u +
    // R gain mn (1 - e2)^bp + (1 - gain)(C + R mn)   (e2 < 1)
    const double mn = k.b_minlum, gain = k.b_gain;
    cc->b_bk_a = (float)(-1.0 / R), cc->b_bk_b = (float)((R + C) / R);
    cc->b_bk_c = (float)(R * gain * mn), cc->b_bk_d = (float)((1.0 - gain) * (C + R * mn));
  }
  cc->n_peak = k.n_peak, cc->n_rein_off = k.n_rein_off, cc->n_rein_scale = k.n_rein_scale;
  cc->n_hable_inv = k.n_hable_inv, cc->n_mob_j = k.n_mob_j, cc->n_mob_a = k.n_mob_a, cc->n_mob_b = k.n_mob_b;
  cc->n_mob_scale = k.n_mob_scale;
}

// the per-frame record for a smoothed peak (units of 100 nits) and average
// PQ level: the constants of the launch's curve family (the others stay
// zero; each family's double-precision setup is several pow calls, and the
// records of a launch are made in one block on the critical path)
__host__ __device__ inline void curve_for_peak(const PeakModel& m, double peak, double avg_pq, CurveConsts* cc) {
  CurveConsts plain{};
  if (m.family == 7) bt2390_consts(peak, m.t_white, m.t_black, m.knee_off, &plain, m.pq);
  else if (m.family == 8) spline_consts(peak, avg_pq, m.contrast, m.t_white, m.t_black, &plain, m.pq);
  else lp_norm_consts(peak, m.tm_param, m.t_white, &plain);
  curve_fast(plain, cc);
  cc->x_peak = peak, cc->x_avg = avg_pq;
}

// the frame's peak (units of 100 nits, as vf_tonemap's peak) from the
// smoothed PQ maximum, clamped to [min_peak, static peak]
__host__ __device__ inline double peak_of(const PeakModel& m, double max_pq) {
  double peak = hd_pq_eotf(max_pq) * 100.0;
  if (peak < m.min_peak) peak = m.min_peak;  // minimum_peak x the target white
  if (peak > m.static_peak) peak = m.static_peak;
  return peak;
}

// one frame into the smoothing state (max, avg, frames; the caller sets
// .peak = peak_of(m, .max) for the last frame).  IIR with coefficient
// m.iir_a = 1 - exp(-1 / smoothing_period) on the PQ-domain frame max and average; a
// scene change (frame-average jump of scene_low .. scene_high % PQ) bypasses
// it progressively (smoothstep); negative thresholds turn that off
__host__ __device__ inline void peak_iir_step(PeakState* s, const PeakModel& m, double fmax, double favg) {
  if (s->frames == 0) {
    s->max = fmax, s->avg = favg;
  } else {
    const double a = m.iir_a;
    const double d = fabs(favg - s->avg) * 100.0;
    double t = 0.0;
    if (m.scene_low >= 0.0 && m.scene_high >= 0.0)
      t = m.scene_high > m.scene_low ? (d - m.scene_low) / (m.scene_high - m.scene_low) : (d >= m.scene_low ? 1.0 : 0.0);
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    const double w = a + (1.0 - a) * t * t * (3.0 - 2.0 * t);
    s->max += w * (fmax - s->max);
    s->avg += w * (favg - s->avg);
  }
  s->frames++;
}

}  // namespace h2s
