// h2s_api.hip — the C-ABI (include/h2s.h): contexts, parameter resolution,
// LUT upload, frame validation, host staging and kernel timing.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#define H2S_PRIVATE_TEST_HOOKS
#include "../../include/h2s.h"
#include "h2s_device.h"
#include "h2s_peak.h"

namespace h2s {
hipError_t launch_process(const KParams& P, bool vec, bool out8, hipStream_t s);
hipError_t launch_debug(const KParams& P, int stage, float* out, hipStream_t s);
bool fast_supported(int tonemap);
hipError_t launch_fast(const FastParams& F, int trc, int tm, int desat, int lp, hipStream_t s, int dbg = 0);
hipError_t launch_process_c444(const KParams& P, bool out8, hipStream_t s);
hipError_t launch_chroma_bicubic(const KParams& P, const float* wx7, const float* wy8, bool out8, hipStream_t s);
hipError_t build_lut_yuv(const float4* rgb, float* yuv, int n, const YuvLutConsts& K, hipStream_t st);
hipError_t build_lut8x(const float4* lut, int n, unsigned* out, hipStream_t s);
hipError_t launch_resize_u8(const uint8_t* src, int sw, int sh, long long sls, long long sfp, uint8_t* dst, int ow,
                            int oh, long long dls, long long dfp, const float* wx, const int* sx, const float* wy,
                            const int* sy, int T, int nframes, hipStream_t s);
hipError_t launch_yuv8_rgb24(const uint8_t* yp, long long yls, const uint8_t* up, const uint8_t* vp, long long cls,
                             long long yuv_fp, int w, int h, uint8_t* rgb, long long rls, long long rgb_fp,
                             const uint8_t* glut, int nframes, hipStream_t s);
hipError_t launch_peak_stats(const KParams& P, float2* partial, const PeakTail& T, hipStream_t s);
hipError_t launch_peak_curves(double2* fstat, int n, const PeakModel& M, PeakState* st, CurveConsts* out,
                              hipStream_t s);
}  // namespace h2s

using h2s::FastParams;
using h2s::KParams;

namespace {
thread_local std::string g_err;  // errors with no context
constexpr int kEvRing = 256;
constexpr int kMaxChunks = 8;  // host-frame pipeline depth (chunks per call)
}  // namespace

struct h2s_ctx {
  int device = 0;
  h2s_params params{};
  bool params_set = false;
  KParams k{};  // resolved constants (pointers filled per call)
  float4* d_lut = nullptr;
  int lut_n = 0;
  float* d_lut_yuv = nullptr;  // lattice pre-multiplied into output code space (3 floats/point)
  float lut_yuv_scale = -1.0f;  // quantiser scale it was built for (-1 = stale)
  int lut_yuv_rgb = 0;          // 1: it holds plain R'G'B' records (libplacebo rgba8 form)
  unsigned* d_lut8x = nullptr;  // libplacebo branch: lut3d's 8-bit output per rgba code triple (2^24, 64 MiB)
  bool lut8x_ok = false;        // built for the current lattice
  bool fast_enabled = true;
  bool lp_exact = false;  // H2S_OPT_LP_EXACT
  int peak_blocks = h2s::PEAK_BLOCKS;   // H2S_OPT_TEST_PEAK_BLOCKS (private A/B hook)
  int peak_form = 0;      // H2S_OPT_TEST_PEAK_FORM (private A/B hook)
  bool serial_host = false;  // H2S_HOST_SERIAL=1: one H2D, kernel, D2H per call (no chunk pipeline)
  int tiles_per_block = 8;  // k_tile: tiles one block walks (H2S_TILES_PER_BLOCK overrides, 1..64)
  uint16_t* d_eq = nullptr;
  float4* d_pq = nullptr;  // PQ EOTF cubic segments (fast path)
  float4* d_hlg = nullptr; // HLG inverse-OETF cubic segments (fast path, CPU chain)
  float4* d_pqi = nullptr; // PQ inverse EOTF cubic segments (fast path, lp_tone IPT)
  void* d_stage = nullptr;
  size_t stage_bytes = 0;
  void* d_prev = nullptr;  // preview scratch
  size_t prev_bytes = 0;
  // dynamic peak (params.peak_detect), all on the device: statistics ->
  // per-frame (max, avg) -> IIR + curve records -> conversion, queued on the
  // caller's stream with no host round trip (h2s_peak.h)
  void* d_stats = nullptr;       // per-block partials, then (percentile model) histograms
  int stats_nf = 0;   // frames d_stats is laid out for (frame_stats)
  double2* d_fstat = nullptr;    // per frame: the statistic, then the smoothed (max, avg) its curve uses
  size_t fstat_cap = 0;
  h2s::CurveConsts* d_curve = nullptr;    // one curve record per frame of a dynamic-peak launch
  size_t curve_cap = 0;
  h2s::PeakState* d_pk = nullptr;         // [0] the smoothing state; [1] a preview's saved copy of it
  hipEvent_t peak_ev = nullptr;           // after the last launch that used the buffers above
  bool peak_pending = false;
  // pipelined schedule (run_dynamic_peak_chunked; private A/B hook
  // H2S_OPT_TEST_PEAK_CHUNK, off: measured slower): frames per
  // chunk (0 = one statistics launch, then one conversion launch, all on the
  // caller's stream), the statistics stream and a second conversion stream,
  // events: start | end | per-chunk statistics
  int peak_chunk = 0;
  hipStream_t pk_s[2] = {};
  std::vector<hipEvent_t> pk_ev;
  std::string err;
  bool fail_after_launch = false;  // H2S_OPT_TEST_FAIL_AFTER_LAUNCH (private test hook, one call)
  bool timing = false;
  hipEvent_t ev0[kEvRing] = {}, ev1[kEvRing] = {};
  long long ev_count = 0;  // launches recorded since reset
  // host-frame pipeline: H2D, compute and D2H of consecutive chunks on
  // their own streams (two DMA directions overlap the kernel and each other)
  hipStream_t ps[3] = {};
  hipEvent_t pev[2 * kMaxChunks + 2] = {};
  // events recorded after this context's own asynchronous launches, on the
  // streams they went to: set_params / set_lut wait for exactly these (no
  // device-wide synchronisation), then recycle them
  std::vector<hipEvent_t> pend, ev_free;
  hipEvent_t chr_ev = nullptr;   // after the last BICUBIC two-pass launch (d_chr scratch in use)
  // set_params / set_lut copy and (re)allocate on this non-blocking stream
  // (stream-ordered hipMallocAsync / hipFreeAsync for the lattices): no
  // null-stream copy or hipFree, which would wait for the whole device
  hipStream_t aux = nullptr;
  bool chr_pending = false;
  float2* d_chr = nullptr;       // BICUBIC chroma: one frame's per-pixel (Cb, Cr)
  size_t chr_cap = 0;
};

namespace {

int fail(h2s_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  else g_err = msg;
  return code;
}

int hip_fail(h2s_ctx* c, hipError_t e, const char* what) {
  return fail(c, H2S_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) hipSetDevice(prev);
  }
};

// ---- parameter resolution (mirrors vf_tonemap init/filter_frame, zimg,
// vf_eq create_lut; the CPU statement is oracle/h2s_oracle.c resolve()) ----
float hable_h(float in) { return h2s::hd_hable(in); }

double pq_encode_d(double y) { return h2s::hd_pq_encode(y); }

int validate_params(h2s_ctx* c, const h2s_params* p) {
  if (p->transfer_in != H2S_TRC_PQ && p->transfer_in != H2S_TRC_HLG)
    return fail(c, H2S_E_INVALID_ARG, "transfer_in must be PQ or HLG");
  if (p->bits_in != 10 && p->bits_in != 12)
    return fail(c, H2S_E_UNSUPPORTED, "bits_in must be 10 or 12 (yuv420p10le / yuv420p12le)");
  if (p->bits_out != 8 && p->bits_out != 10 && p->bits_out != 12)
    return fail(c, H2S_E_UNSUPPORTED, "bits_out must be 8, 10 or 12");
  if (p->tonemap < H2S_TM_NONE || p->tonemap > H2S_TM_SPLINE)
    return fail(c, H2S_E_INVALID_ARG, "unknown tonemap operator");
  if (p->tonemap == H2S_TM_SPLINE && !isnan(p->tm_param) && !(p->tm_param >= 0.0 && p->tm_param <= 1.5))
    return fail(c, H2S_E_INVALID_ARG, "spline contrast (tm_param) must be in [0, 1.5]");
  if (p->mode != H2S_MODE_COMPAT8 && p->mode != H2S_MODE_NATIVE)
    return fail(c, H2S_E_INVALID_ARG, "mode must be COMPAT8 or NATIVE");
  if (p->desat_luma < 0 || p->desat_luma > 2) return fail(c, H2S_E_INVALID_ARG, "unknown desat_luma");
  if (!(p->gamma > 0) || !isfinite(p->gamma)) return fail(c, H2S_E_INVALID_ARG, "gamma must be > 0");
  if (!(p->npl > 0) || !isfinite(p->npl)) return fail(c, H2S_E_INVALID_ARG, "npl must be > 0");
  if (!(p->desat >= 0)) return fail(c, H2S_E_INVALID_ARG, "desat must be >= 0");
  if (p->chroma_filter != H2S_CHROMA_BOX && p->chroma_filter != H2S_CHROMA_BICUBIC)
    return fail(c, H2S_E_INVALID_ARG, "unknown chroma_filter");
  if (p->dither != H2S_DITHER_NONE && p->dither != H2S_DITHER_ORDERED)
    return fail(c, H2S_E_INVALID_ARG, "unknown dither");
  if (p->expand != H2S_EXPAND_SHIFT && p->expand != H2S_EXPAND_REPLICATE)
    return fail(c, H2S_E_INVALID_ARG, "unknown expand");
  if (p->chroma_edge < H2S_EDGE_ZIMG || p->chroma_edge > H2S_EDGE_MIRROR)
    return fail(c, H2S_E_INVALID_ARG, "unknown chroma_edge");
  if (p->lut_input != H2S_LUT_IN_FLOAT && p->lut_input != H2S_LUT_IN_RGB48)
    return fail(c, H2S_E_INVALID_ARG, "unknown lut_input");
  if (p->pipeline < H2S_PIPE_AUTO || p->pipeline > H2S_PIPE_LIBPLACEBO)
    return fail(c, H2S_E_INVALID_ARG, "unknown pipeline");
  if (p->lp_tone != H2S_LP_TONE_IPT && p->lp_tone != H2S_LP_TONE_MAX_RGB)
    return fail(c, H2S_E_INVALID_ARG, "unknown lp_tone");
  if (p->pipeline == H2S_PIPE_LIBPLACEBO && (p->tonemap < H2S_TM_REINHARD || p->tonemap > H2S_TM_SPLINE))
    return fail(c, H2S_E_UNSUPPORTED,
                "libplacebo pipeline: the reference's operators are reinhard, mobius, hable, bt.2390 and spline");
  if (!isnan(p->knee_offset) && !(p->knee_offset >= 0.5 && p->knee_offset <= 2.0))
    return fail(c, H2S_E_INVALID_ARG, "knee_offset must be in [0.5, 2] (libplacebo's range)");
  if (!isnan(p->target_white) && !(p->target_white > 0 && isfinite(p->target_white)))
    return fail(c, H2S_E_INVALID_ARG, "target_white must be > 0");
  if (!isnan(p->target_black) && !(p->target_black >= 0 && isfinite(p->target_black)))
    return fail(c, H2S_E_INVALID_ARG, "target_black must be >= 0");
  if (!isnan(p->target_black) && !isnan(p->target_white) && !(p->target_black < p->target_white))
    return fail(c, H2S_E_INVALID_ARG, "target_black must be below target_white");
  if (p->lp_range != H2S_LP_RANGE_FULL && p->lp_range != H2S_LP_RANGE_LIMITED)
    return fail(c, H2S_E_INVALID_ARG, "unknown lp_range");
  if (p->lp_dither != H2S_LP_DITHER_NONE && p->lp_dither != H2S_LP_DITHER_ORDERED)
    return fail(c, H2S_E_INVALID_ARG, "unknown lp_dither");
  if (p->lp_p010 != H2S_LP_P010_KEEP && p->lp_p010 != H2S_LP_P010_TRUNCATE)
    return fail(c, H2S_E_INVALID_ARG, "unknown lp_p010");
  // vf_libplacebo's option ranges (smoothing_period 0..1000, scene thresholds
  // -1..100 (negative: scene detection off), percentile 0..100, minimum_peak 0..100)
  if (!isnan(p->pd_smoothing) && !(p->pd_smoothing >= 0.0 && p->pd_smoothing <= 1000.0))
    return fail(c, H2S_E_INVALID_ARG, "pd_smoothing must be in [0, 1000] frames");
  if (!isnan(p->pd_scene_low) && !(p->pd_scene_low >= -1.0 && p->pd_scene_low <= 100.0))
    return fail(c, H2S_E_INVALID_ARG, "pd_scene_low must be in [-1, 100]");
  if (!isnan(p->pd_scene_high) && !(p->pd_scene_high >= -1.0 && p->pd_scene_high <= 100.0))
    return fail(c, H2S_E_INVALID_ARG, "pd_scene_high must be in [-1, 100]");
  if (!isnan(p->pd_percentile) && !(p->pd_percentile > 0.0 && p->pd_percentile <= 100.0))
    return fail(c, H2S_E_INVALID_ARG, "pd_percentile must be in (0, 100]");
  if (!isnan(p->pd_min_peak) && !(p->pd_min_peak >= 0.0 && p->pd_min_peak <= 100.0))
    return fail(c, H2S_E_INVALID_ARG, "pd_min_peak must be in [0, 100]");
  return 0;
}

// the per-frame curve constants (BT.2390, spline, libplacebo's NORM curves)
// and their folded fast-kernel form are h2s_peak.h's host/device functions

// IPT-PQ matrices (h2s_lp_tone IPT), in double: BT.2020 RGB -> XYZ from the
// primaries and D65 white, XYZ -> LMS by the Hunt-Pointer-Estevez matrix of
// IPT (D65-normalised: neutral L = M = S = Y), and the inverse.  Keeping P and
// T reduces to L'M'S' += I' - I (the inverse IPT matrix has an I column of 1)
static void inv3(const double m[3][3], double o[3][3]) {
  const double d = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                   m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      o[i][j] = (m[(j + 1) % 3][(i + 1) % 3] * m[(j + 2) % 3][(i + 2) % 3] -
                 m[(j + 1) % 3][(i + 2) % 3] * m[(j + 2) % 3][(i + 1) % 3]) / d;
}

static void ipt_matrices(double r2l[9], double l2r[9]) {
  const double prim[3][2] = {{0.708, 0.292}, {0.170, 0.797}, {0.131, 0.046}}, wx = 0.3127, wy = 0.3290;
  double xyz[3][3], xyzi[3][3];
  for (int k = 0; k < 3; k++) {
    xyz[0][k] = prim[k][0] / prim[k][1];
    xyz[1][k] = 1.0;
    xyz[2][k] = (1.0 - prim[k][0] - prim[k][1]) / prim[k][1];
  }
  inv3(xyz, xyzi);
  const double w[3] = {wx / wy, 1.0, (1.0 - wx - wy) / wy};
  for (int k = 0; k < 3; k++) {
    const double sk = xyzi[k][0] * w[0] + xyzi[k][1] * w[1] + xyzi[k][2] * w[2];
    for (int i = 0; i < 3; i++) xyz[i][k] *= sk;                       // RGB -> XYZ
  }
  const double hpe[3][3] = {{0.4002, 0.7076, -0.0808}, {-0.2263, 1.1653, 0.0457}, {0.0, 0.0, 0.9182}};
  double rl[3][3], lr[3][3];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) rl[i][k] = hpe[i][0] * xyz[0][k] + hpe[i][1] * xyz[1][k] + hpe[i][2] * xyz[2][k];
  inv3(rl, lr);
  for (int i = 0; i < 9; i++) r2l[i] = rl[i / 3][i % 3], l2r[i] = lr[i / 3][i % 3];
}

void resolve(const h2s_params* p, KParams* k, std::vector<uint16_t>* eq) {
  memset(k, 0, sizeof(*k));
  // S1 zimg: depth conversion (limited range), BT.2020-NCL matrix, scale
  const int sh = p->bits_in - 8;
  k->y_scale = (float)(1.0 / (219 << sh));
  k->y_off = (float)(-(double)(16 << sh) / (219 << sh));
  k->c_scale = (float)(1.0 / (224 << sh));
  k->c_off = (float)(-(double)(128 << sh) / (224 << sh));
  const double kr = 0.2627, kb = 0.0593, kg = 1.0 - kr - kb;
  k->m_rcr = (float)(2.0 * (1.0 - kr));
  k->m_gcb = (float)(-2.0 * kb * (1.0 - kb) / kg);
  k->m_gcr = (float)(-2.0 * kr * (1.0 - kr) / kg);
  k->m_bcb = (float)(2.0 * (1.0 - kb));
  k->transfer = p->transfer_in;
  k->lin_scale = (float)((p->transfer_in == H2S_TRC_HLG ? 1000.0 : 10000.0) / p->npl);

  // S2 vf_tonemap init defaults
  double param = p->tm_param;
  switch (p->tonemap) {
    case H2S_TM_GAMMA:
      if (isnan(param)) param = 1.8;
      break;
    case H2S_TM_REINHARD:
      if (!isnan(param)) param = (1.0 - param) / param;
      break;
    case H2S_TM_MOBIUS:
      if (isnan(param)) param = 0.3;
      break;
  }
  if (isnan(param)) param = 1.0;
  // ff_determine_signal_peak; trc at tonemap's input is linear -> 10.0
  double peak = p->peak;
  if (!(peak > 0)) {
    peak = 0;
    if (p->maxcll > 0) peak = p->maxcll / 100.0;
    if (!(peak > 0) && p->mastering_max > 0) peak = p->mastering_max / 100.0;
    if (!(peak > 0)) peak = 10.0;
  }
  k->tonemap = p->tonemap;
  k->desat_on = p->desat > 0 ? 1 : 0;
  k->desat = (float)p->desat;
  switch (p->desat_luma) {
    case H2S_DESAT_LUMA_BT2020: k->lr = 0.2627f, k->lg = 0.6780f, k->lb = 0.0593f; break;
    case H2S_DESAT_LUMA_BT709: k->lr = 0.2126f, k->lg = 0.7152f, k->lb = 0.0722f; break;
    default: k->lr = 1.0f, k->lg = 1.0f, k->lb = 1.0f;
  }
  k->lin_k = (float)(param / peak);
  k->gam_inv_peak = (float)(1.0 / peak);
  k->gam_inv_param = (float)(1.0 / param);
  k->gam_low_k = (float)(pow(0.05 / peak, 1.0 / param) / 0.05);
  k->clip_k = (float)param;
  k->hable_peak_inv = 1.0f / hable_h((float)peak);
  k->rein_p = (float)param;
  k->rein_k = (float)((peak + param) / peak);
  {
    const float j = (float)param;
    const float a = (float)(-j * j * (peak - 1.0f) / (j * j - 2.0f * j + peak));
    const float b = (float)((j * j - 2.0f * j * peak + peak) / fmax(peak - 1.0f, 1e-6));
    k->mob_j = j, k->mob_a = a, k->mob_b = b;
    k->mob_k = (b * b + 2.0f * b * j + j * j) / (b - a);
  }
  k->peak = peak;
  k->x_peak = peak, k->x_avg = 0.0, k->x_npl = p->npl, k->x_tm_param = p->tm_param, k->x_sh = p->bits_in - 8;
  // pipeline and SDR target (oracle resolve: the CPU chain's curve output is
  // relative to npl with no black; libplacebo targets PL_COLOR_SDR_WHITE =
  // 203 nits at PL_COLOR_SDR_CONTRAST = 1000:1)
  k->pipe = p->pipeline != H2S_PIPE_AUTO ? p->pipeline
                                         : (p->tonemap == H2S_TM_BT2390 || p->tonemap == H2S_TM_SPLINE ? h2s::PIPE_LIBPLACEBO
                                                                                                      : h2s::PIPE_CPU);
  const bool lp = k->pipe == h2s::PIPE_LIBPLACEBO;
  k->rgba8 = lp && p->lut_enabled ? 1 : 0;
  k->lp_ipt = lp && p->lp_tone == H2S_LP_TONE_IPT ? 1 : 0;
  // libplacebo stage options (ABI v3): range=tv on the rgba output, the
  // download's dither, the 12-bit input through format=p010
  const bool lim = lp && p->lp_range == H2S_LP_RANGE_LIMITED;
  k->lp_qs = lim ? 219.0f : 255.0f;
  k->lp_qo = lim ? 16.0f : 0.0f;
  k->lp_dith = lp && p->lp_dither == H2S_LP_DITHER_ORDERED ? 1 : 0;
  k->in_mask = lp && p->lp_p010 == H2S_LP_P010_TRUNCATE && p->bits_in == 12 ? 0xFFFCu : 0xFFFFu;
  ipt_matrices(k->ipt_r2l, k->ipt_l2r);
  k->t_white = isnan(p->target_white) ? (lp ? 203.0 : p->npl) : p->target_white;
  k->t_black = isnan(p->target_black) ? (lp ? k->t_white / 1000.0 : 0.0) : p->target_black;
  // peak_detect=1: vf_libplacebo's option defaults (smoothing_period 100,
  // scene_threshold_low / high 5.5 / 10, percentile 99.995, minimum_peak 1
  // x the SDR white); PARITY UNPINNED
  k->pd_smoothing = isnan(p->pd_smoothing) ? 100.0 : p->pd_smoothing;
  k->pd_scene_low = isnan(p->pd_scene_low) ? 5.5 : p->pd_scene_low;
  k->pd_scene_high = isnan(p->pd_scene_high) ? 10.0 : p->pd_scene_high;
  k->pd_percentile = isnan(p->pd_percentile) ? 99.995 : p->pd_percentile;
  k->pd_min = (isnan(p->pd_min_peak) ? 1.0 : p->pd_min_peak) * k->t_white / 100.0;
  k->knee_off = isnan(p->knee_offset) ? 1.0 : p->knee_offset;
  {
    const double lb = pow(k->t_black / k->t_white, 1.0 / 2.4), a = pow(1.0 - lb, 2.4);
    k->enc_ainv = (float)(1.0 / a);
    k->enc_a = (float)a;
    k->enc_b = (float)(lb / (1.0 - lb));
  }
  h2s::bt2390_consts(peak, k->t_white, k->t_black, k->knee_off, k, h2s::pq_refs(k->t_white, k->t_black));
  k->sp_contrast = isnan(p->tm_param) ? 0.5f : (float)p->tm_param;
  h2s::spline_consts(peak, 0.0, (double)k->sp_contrast, k->t_white, k->t_black, k, h2s::pq_refs(k->t_white, k->t_black));
  k->npl_1e4 = (float)(p->npl / 10000.0);
  k->e4_npl = (float)(10000.0 / k->t_white);
  k->ipt_npl = p->npl / 10000.0, k->ipt_os = 10000.0 / k->t_white, k->ipt_tw = k->t_white / 10000.0;
  k->lp_norm = lp && p->tonemap >= H2S_TM_REINHARD && p->tonemap <= H2S_TM_MOBIUS ? 1 : 0;
  k->n_nw = (float)(p->npl / k->t_white);
  h2s::lp_norm_consts(peak, p->tm_param, k->t_white, k);
  // closed-form gamut step (lut_enabled = 0), tools/generate_lut.py:36-40
  const double m[9] = {1.6604910021, -0.5876411388, -0.0728498633, -0.1245504745, 1.1328998971,
                       -0.0083494226, -0.0181507634, -0.1005788980, 1.1187296614};
  for (int i = 0; i < 9; i++) k->m709[i] = (float)m[i];
  k->lut_enabled = p->lut_enabled ? 1 : 0;
  // S6 BT.709 limited-range Y'CbCr rows
  const double r709 = 0.2126, g709 = 0.7152, b709 = 0.0722;
  k->k709[0] = (float)r709, k->k709[1] = (float)g709, k->k709[2] = (float)b709;
  k->kcb[0] = (float)(-r709 / 1.8556), k->kcb[1] = (float)(-g709 / 1.8556), k->kcb[2] = (float)(0.9278 / 1.8556);
  k->kcr[0] = (float)(0.7874 / 1.5748), k->kcr[1] = (float)(-g709 / 1.5748), k->kcr[2] = (float)(-b709 / 1.5748);
  // quantisation depth (oracle resolve): eq's yuv420p (compat8) or bits_out
  // (native; the libplacebo rgba frame with gamma 1 has no eq to pass)
  const int q = p->mode == H2S_MODE_NATIVE || (k->rgba8 && p->gamma == 1.0) ? p->bits_out : 8;
  k->qmax = (1 << q) - 1;
  k->qscale = (float)(1 << (q - 8));
  k->shift_out = p->bits_out - q;
  k->dither = p->dither == H2S_DITHER_ORDERED && q == 8 ? 1 : 0;
  k->expand_rep = p->expand == H2S_EXPAND_REPLICATE ? 1 : 0;
  k->chroma_edge = p->chroma_edge;
  k->lut_in16 = p->lut_input == H2S_LUT_IN_RGB48 && !lp ? 1 : 0;  // the CPU chain's S3 -> S4
  // S7 vf_eq create_lut, generalised to 2^q entries
  const int qn = 1 << q;
  eq->assign(qn, 0);
  bool ident = true;
  const double g = 1.0 / p->gamma;
  for (int i = 0; i < qn; i++) {
    double v = i / (double)(qn - 1);
    uint16_t o;
    if (v <= 0.0) {
      o = 0;
    } else {
      v = pow(v, g);
      o = v >= 1.0 ? (uint16_t)(qn - 1) : (uint16_t)(int)((double)qn * v);
    }
    (*eq)[i] = o;
    if (o != i) ident = false;
  }
  k->eq_identity = ident ? 1 : 0;
}

// ST 2084 inverse EOTF (y = luminance / 10000 -> E) as PQI_NSEG cubic
// segments for the tile kernel's IPT form (h2s_tile.h pqi): segment s covers
// y = 2^e (1 + j/8 + t), e = PQI_OCT0 + s/8, j = s%8, t in [0, 1/8), read from
// the float's exponent and top three mantissa bits; the cubic in t through
// the exact (double) encode at the 4 Chebyshev nodes (relative error <=
// 1.5e-7 with float32 coefficients).  Entry 0 is the constant PQ(0), read for
// y <= 0 and for y below the first octave (2^-64, 1e-15 nits: PQ within 3e-7
// of PQ(0)); segment s is entry 1 + s (PQI_NTAB entries)
static void solve_cubic(const double t[4], const double y[4], double c[4]) {
  double A[4][5];
  for (int k = 0; k < 4; k++) {
    for (int j = 0; j < 4; j++) A[k][j] = pow(t[k], j);
    A[k][4] = y[k];
  }
  for (int col = 0; col < 4; col++) {
    int piv = col;
    for (int r = col + 1; r < 4; r++)
      if (fabs(A[r][col]) > fabs(A[piv][col])) piv = r;
    for (int j = 0; j < 5; j++) std::swap(A[col][j], A[piv][j]);
    for (int r = 0; r < 4; r++) {
      if (r == col) continue;
      const double fct = A[r][col] / A[col][col];
      for (int j = col; j < 5; j++) A[r][j] -= fct * A[col][j];
    }
  }
  for (int k = 0; k < 4; k++) c[k] = A[k][4] / A[k][k];
}

void build_pqi_table(std::vector<float4>* out) {
  constexpr int K = h2s::PQI_PER_OCT;
  out->resize(h2s::PQI_NTAB);
  (*out)[0] = make_float4(0.0f, 0.0f, 0.0f, (float)pq_encode_d(0.0));
  double t[4];
  for (int k = 0; k < 4; k++) t[k] = (1.0 - cos((2 * k + 1) * M_PI / 8.0)) / 2.0 / K;
  for (int sg = 0; sg < h2s::PQI_NSEG; sg++) {
    const double base = ldexp(1.0, h2s::PQI_OCT0 + sg / K);
    double y[4], c[4];
    for (int k = 0; k < 4; k++) y[k] = pq_encode_d(base * (1.0 + (double)(sg % K) / K + t[k]));
    solve_cubic(t, y, c);
    (*out)[1 + sg] = make_float4((float)c[3], (float)c[2], (float)c[1], (float)c[0]);
  }
}

// PQ EOTF x scale as PQ_NSEG cubic segments: per segment, the cubic through
// the exact (double) EOTF at the 4 Chebyshev nodes of the segment.  Measured
// max relative error 1.2e-7 for E > 0.05 (float32 evaluation).
// cubic segments of f over E in [i, i+1) / PQ_SEG, i < PQ_NSEG, interpolating
// f at the four Chebyshev nodes of each segment (k_tile's pq_z layout)
template <class Fn>
static void build_seg_table(const Fn& eotf, std::vector<float4>* out) {
  double t[4];
  for (int k = 0; k < 4; k++) t[k] = (1.0 - cos((2 * k + 1) * M_PI / 8.0)) / 2.0;
  out->resize(h2s::PQ_NSEG);
  for (int i = 0; i < h2s::PQ_NSEG; i++) {
    // solve the 4x4 Vandermonde system A c = y (c = c0..c3) by Gaussian elimination
    double A[4][5];
    for (int k = 0; k < 4; k++) {
      for (int j = 0; j < 4; j++) A[k][j] = pow(t[k], j);
      A[k][4] = eotf((i + t[k]) / h2s::PQ_SEG);
    }
    for (int col = 0; col < 4; col++) {
      int piv = col;
      for (int r = col + 1; r < 4; r++)
        if (fabs(A[r][col]) > fabs(A[piv][col])) piv = r;
      for (int j = 0; j < 5; j++) std::swap(A[col][j], A[piv][j]);
      for (int r = 0; r < 4; r++) {
        if (r == col) continue;
        const double fct = A[r][col] / A[col][col];
        for (int j = col; j < 5; j++) A[r][j] -= fct * A[col][j];
      }
    }
    double c[4];
    for (int k = 0; k < 4; k++) c[k] = A[k][4] / A[k][k];
    if (i == 0) c[0] = 0.0;  // E = 0 maps to exactly 0, as zimg's x > 0 test
    (*out)[i] = make_float4((float)c[3], (float)c[2], (float)c[1], (float)c[0]);
  }
}

void build_pq_table(double scale, std::vector<float4>* out) {
  const double m1 = 2610.0 / 16384, m2 = 2523.0 / 32, c1 = 3424.0 / 4096, c2 = 2413.0 / 128, c3 = 2392.0 / 128;
  build_seg_table([&](double e) {
    if (!(e > 0)) return 0.0;
    const double xp = pow(e, 1.0 / m2);
    const double num = fmax(xp - c1, 0.0), den = c2 - c3 * xp;
    return den > 0 ? pow(num / den, 1.0 / m1) * scale : HUGE_VAL;
  }, out);
}

// zimg arib_b67_inverse_oetf (k_tile's HLG input on the CPU chain; the OOTF
// follows in the kernel): E^2 / 3 up to 1/2, (exp((E - c) / a) + b) / 12
// above; 1/2 is a segment boundary, so every segment interpolates one smooth
// branch (the quadratic one exactly)
void build_hlg_table(std::vector<float4>* out) {
  const double a = 0.17883277, b = 0.28466892, c = 0.55991073;
  build_seg_table([&](double e) {
    if (!(e > 0)) return 0.0;
    return e <= 0.5 ? e * e / 3.0 : (exp((e - c) / a) + b) / 12.0;
  }, out);
}

bool aligned(const void* p, long long a) { return ((uintptr_t)p % (uintptr_t)a) == 0; }

int check_frames(h2s_ctx* c, const h2s_frames* f, int bits, const char* which) {
  if (!f) return fail(c, H2S_E_INVALID_ARG, std::string(which) + " frames is NULL");
  if (f->width <= 0 || f->height <= 0) return fail(c, H2S_E_INVALID_ARG, std::string(which) + ": empty frame");
  if ((f->width & 1) || (f->height & 1))
    return fail(c, H2S_E_UNSUPPORTED, std::string(which) + ": 4:2:0 frames need even width and height");
  if (f->bits != bits)
    return fail(c, H2S_E_INVALID_ARG,
                std::string(which) + ": bits " + std::to_string(f->bits) + " != params " + std::to_string(bits));
  if (f->location != H2S_LOC_DEVICE && f->location != H2S_LOC_HOST)
    return fail(c, H2S_E_INVALID_ARG, std::string(which) + ": bad location");
  const int bps = bits == 8 ? 1 : 2;
  const long long rowb[3] = {(long long)f->width * bps, (long long)f->width / 2 * bps, (long long)f->width / 2 * bps};
  for (int p = 0; p < 3; p++) {
    if (!f->data[p]) return fail(c, H2S_E_INVALID_ARG, std::string(which) + ": NULL plane");
    if (f->linesize[p] < rowb[p])
      return fail(c, H2S_E_INVALID_ARG, std::string(which) + ": linesize smaller than a row");
    if (bps == 2 && ((f->linesize[p] & 1) || !aligned(f->data[p], 2)))
      return fail(c, H2S_E_INVALID_ARG, std::string(which) + ": 16-bit planes must be 2-byte aligned");
  }
  return 0;
}

// vector path needs 16-B luma / 8-B chroma alignment of every row start
bool vec_ok(const h2s_frames* f, bool out8) {
  const long long ay = out8 ? 8 : 16, ac = out8 ? 4 : 8;
  const long long a[3] = {ay, ac, ac};
  for (int p = 0; p < 3; p++)
    if (!aligned(f->data[p], a[p]) || f->linesize[p] % a[p] || f->frame_pitch[p] % a[p]) return false;
  return true;
}

// tile kernel: at least one 64-pixel tile, every row start 16-B aligned (8-B
// for 8-bit chroma output)
bool tile_ok(const h2s_frames* in, const h2s_frames* out, bool out8, int tw) {
  if (in->width < tw) return false;  // width % tw columns go to k_process (launch_chain)
  for (int p = 0; p < 3; p++) {
    if (!aligned(in->data[p], 16) || in->linesize[p] % 16 || in->frame_pitch[p] % 16) return false;
    const long long a = out8 ? (p ? 8 : 8) : 16;
    if (!aligned(out->data[p], a) || out->linesize[p] % a || out->frame_pitch[p] % a) return false;
  }
  return true;
}

size_t frame_bytes(const h2s_frames* f) {
  const size_t bps = f->bits == 8 ? 1 : 2;
  return (size_t)f->width * f->height * bps * 3 / 2;
}

// tight device copy descriptor laid out in `base`
h2s_frames tight(const h2s_frames* f, void* base) {
  h2s_frames t = *f;
  const long long bps = f->bits == 8 ? 1 : 2;
  const long long ysz = (long long)f->width * f->height * bps, csz = ysz / 4;
  const long long fb = ysz + 2 * csz;
  t.data[0] = base;
  t.data[1] = (uint8_t*)base + ysz;
  t.data[2] = (uint8_t*)base + ysz + csz;
  t.linesize[0] = f->width * bps;
  t.linesize[1] = t.linesize[2] = f->width / 2 * bps;
  t.frame_pitch[0] = t.frame_pitch[1] = t.frame_pitch[2] = fb;
  t.location = H2S_LOC_DEVICE;
  return t;
}

// the whole batch is one contiguous span laid out as tight() describes
bool is_tight(const h2s_frames* f) {
  const long long bps = f->bits == 8 ? 1 : 2;
  const long long ysz = (long long)f->width * f->height * bps, csz = ysz / 4, fb = ysz + 2 * csz;
  return f->linesize[0] == f->width * bps && f->linesize[1] == f->width / 2 * bps &&
         f->linesize[2] == f->width / 2 * bps && f->frame_pitch[0] == fb && f->frame_pitch[1] == fb &&
         f->frame_pitch[2] == fb && (const uint8_t*)f->data[1] == (const uint8_t*)f->data[0] + ysz &&
         (const uint8_t*)f->data[2] == (const uint8_t*)f->data[1] + csz;
}

hipError_t copy_frames(const h2s_frames* dst, const h2s_frames* src, int nframes, hipStream_t s) {
  const long long bps = src->bits == 8 ? 1 : 2;
  if (is_tight(src) && is_tight(dst))  // one DMA for the whole batch
    return hipMemcpyAsync(dst->data[0], src->data[0], (size_t)src->frame_pitch[0] * nframes, hipMemcpyDefault, s);
  for (int fr = 0; fr < nframes; fr++)
    for (int p = 0; p < 3; p++) {
      const long long w = (p ? src->width / 2 : src->width) * bps, h = p ? src->height / 2 : src->height;
      hipError_t e = hipMemcpy2DAsync((uint8_t*)dst->data[p] + fr * dst->frame_pitch[p], dst->linesize[p],
                                      (const uint8_t*)src->data[p] + fr * src->frame_pitch[p], src->linesize[p], w,
                                      h, hipMemcpyDefault, s);
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}

void fill_geometry(KParams* k, const h2s_frames* in, const h2s_frames* out, int nframes) {
  k->W = in->width;
  k->H = in->height;
  k->cw = in->width / 2;
  k->ch = in->height / 2;
  k->ngx = (k->cw + 3) / 4;
  k->nframes = nframes;
  k->total = (long long)nframes * k->ch * k->ngx;
  for (int p = 0; p < 3; p++) {
    k->in[p] = (const uint8_t*)in->data[p];
    k->in_ls[p] = in->linesize[p];
    k->in_fp[p] = in->frame_pitch[p];
    if (out) {
      k->out[p] = (uint8_t*)out->data[p];
      k->out_ls[p] = out->linesize[p];
      k->out_fp[p] = out->frame_pitch[p];
    }
  }
}

}  // namespace

extern "C" {

int h2s_abi_version(void) { return H2S_ABI_VERSION; }

int h2s_abi_minor(void) { return H2S_ABI_MINOR; }

const char* h2s_last_error(const h2s_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

void h2s_params_default(h2s_params* p) {
  if (!p) return;
  memset(p, 0, sizeof(*p));
  // FFMPEG_CONVERT_FILTER defaults (src/utils.py:38-42) with the settings
  // defaults (src/settings.py:10-26: gamma 1.0, tonemapper Mobius) and the
  // GUI's 10-bit output for <=10-bit sources (src/gui.py:1009-1021).
  p->transfer_in = H2S_TRC_PQ;
  p->bits_in = 10;
  p->bits_out = 10;
  p->tonemap = H2S_TM_MOBIUS;
  p->tm_param = NAN;
  p->desat = 2.0;
  p->peak = 0.0;
  p->npl = 100.0;
  p->gamma = 1.0;
  p->lut_enabled = 1;
  p->mode = H2S_MODE_COMPAT8;
  p->desat_luma = H2S_DESAT_LUMA_RGB;
  // [EXT] switches: the round-1 models; pipeline AUTO; libplacebo targets from the branch
  p->chroma_filter = H2S_CHROMA_BOX;
  p->dither = H2S_DITHER_NONE;
  p->expand = H2S_EXPAND_SHIFT;
  p->pipeline = H2S_PIPE_AUTO;
  p->knee_offset = NAN;
  p->target_black = NAN;
  p->target_white = NAN;
  p->chroma_edge = H2S_EDGE_ZIMG;
  p->lut_input = H2S_LUT_IN_FLOAT;
  p->lp_tone = H2S_LP_TONE_IPT;   // libplacebo >= 6 tone-maps in IPT (h2s.h enum h2s_lp_tone)
  p->lp_range = H2S_LP_RANGE_FULL;
  p->lp_dither = H2S_LP_DITHER_NONE;
  p->lp_p010 = H2S_LP_P010_TRUNCATE;   // format=p010,hwupload (src/utils.py:431)
  p->pd_smoothing = p->pd_scene_low = p->pd_scene_high = p->pd_percentile = p->pd_min_peak = NAN;
}

int h2s_create(int device, h2s_ctx** out) {
  if (!out) return fail(nullptr, H2S_E_INVALID_ARG, "out is NULL");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return fail(nullptr, H2S_E_HIP, "no HIP device available");
  if (device < 0 || device >= n) return fail(nullptr, H2S_E_INVALID_ARG, "device ordinal out of range");
  h2s_ctx* c = new (std::nothrow) h2s_ctx();
  if (!c) return fail(nullptr, H2S_E_OOM, "context allocation failed");
  c->device = device;
  h2s_params_default(&c->params);
  if (const char* v = getenv("H2S_HOST_SERIAL")) c->serial_host = atoi(v) != 0;
  if (const char* v = getenv("H2S_TILES_PER_BLOCK")) {
    const int tpb = atoi(v);
    if (tpb >= 1 && tpb <= 64) c->tiles_per_block = tpb;
  }
  *out = c;
  return 0;
}

void h2s_destroy(h2s_ctx* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  hipDeviceSynchronize();
  if (c->aux) {  // the lattices are stream-ordered allocations of the context stream
    if (c->d_lut) hipFreeAsync(c->d_lut, c->aux);
    if (c->d_lut_yuv) hipFreeAsync(c->d_lut_yuv, c->aux);
    if (c->d_lut8x) hipFreeAsync(c->d_lut8x, c->aux);
    hipStreamSynchronize(c->aux);
    hipStreamDestroy(c->aux);
  }
  if (c->d_eq) hipFree(c->d_eq);
  if (c->d_pq) hipFree(c->d_pq);
  if (c->d_hlg) hipFree(c->d_hlg);
  if (c->d_pqi) hipFree(c->d_pqi);
  if (c->d_stage) hipFree(c->d_stage);
  if (c->d_prev) hipFree(c->d_prev);
  if (c->d_stats) hipFree(c->d_stats);
  if (c->d_fstat) hipFree(c->d_fstat);
  if (c->d_curve) hipFree(c->d_curve);
  if (c->d_pk) hipFree(c->d_pk);
  if (c->d_chr) hipFree(c->d_chr);
  if (c->peak_ev) hipEventDestroy(c->peak_ev);
  for (hipEvent_t ev : c->pk_ev) hipEventDestroy(ev);
  for (hipStream_t ps : c->pk_s)
    if (ps) hipStreamDestroy(ps);
  if (c->chr_ev) hipEventDestroy(c->chr_ev);
  for (hipEvent_t ev : c->pend) hipEventDestroy(ev);
  for (hipEvent_t ev : c->ev_free) hipEventDestroy(ev);
  for (int i = 0; i < kEvRing; i++) {
    if (c->ev0[i]) hipEventDestroy(c->ev0[i]);
    if (c->ev1[i]) hipEventDestroy(c->ev1[i]);
  }
  for (hipEvent_t ev : c->pev)
    if (ev) hipEventDestroy(ev);
  for (hipStream_t ps : c->ps)
    if (ps) hipStreamDestroy(ps);
  delete c;
}

// set_params / set_lut rewrite device tables that this context's queued
// kernels may still read: wait for the events recorded after its own
// launches (include/h2s.h), not for the device
static int drain_launches(h2s_ctx* c) {
  hipError_t e = hipSuccess;
  for (hipEvent_t ev : c->pend) {
    const hipError_t r = hipEventSynchronize(ev);
    if (e == hipSuccess) e = r;
    c->ev_free.push_back(ev);
  }
  c->pend.clear();
  if (e != hipSuccess) return hip_fail(c, e, "draining queued launches");
  return 0;
}

static int aux_stream(h2s_ctx* c, hipStream_t* out) {
  if (!c->aux) {
    hipError_t e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking);
    if (e != hipSuccess) {
      c->aux = nullptr;
      return hip_fail(c, e, "table stream");
    }
  }
  *out = c->aux;
  return 0;
}

// host -> device table copy on the context's own stream, waited for there
static hipError_t table_copy(h2s_ctx* c, void* dst, const void* src, size_t bytes) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->aux);
  return e == hipSuccess ? hipStreamSynchronize(c->aux) : e;
}

static int note_launch(h2s_ctx* c, hipStream_t s);

// an error exit of h2s_process after work was queued on s: record the launch
// event anyway, so that a later set_params / set_lut still waits for that work
// before rewriting the tables it reads (include/h2s.h); if even the event
// cannot be recorded, wait for the stream.  The caller's error stays the one
// reported.
static int queued_exit(h2s_ctx* c, hipStream_t s, int rc) {
  const std::string msg = c->err;
  if (note_launch(c, s) != 0) (void)hipStreamSynchronize(s);
  c->err = msg;
  return rc;
}

// record that this context queued work on stream s (after the launches)
static int note_launch(h2s_ctx* c, hipStream_t s) {
  if (c->pend.size() >= 32) {   // recycle the events that have completed
    size_t j = 0;
    for (size_t i = 0; i < c->pend.size(); i++) {
      if (hipEventQuery(c->pend[i]) == hipSuccess) c->ev_free.push_back(c->pend[i]);
      else c->pend[j++] = c->pend[i];
    }
    c->pend.resize(j);
  }
  hipEvent_t ev = nullptr;
  if (!c->ev_free.empty()) {
    ev = c->ev_free.back();
    c->ev_free.pop_back();
  } else {
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "launch event");
  }
  hipError_t e = hipEventRecord(ev, s);
  if (e != hipSuccess) {
    c->ev_free.push_back(ev);
    return hip_fail(c, e, "launch event");
  }
  c->pend.push_back(ev);
  return 0;
}

int h2s_set_lut(h2s_ctx* c, const float* rgb, int n) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  if (!rgb || n < 2 || n > 256) return fail(c, H2S_E_INVALID_ARG, "LUT size must be in [2, 256]");
  DeviceGuard g(c->device);
  if (int rc = drain_launches(c)) return rc;
  const size_t cnt = (size_t)n * n * n;
  std::vector<float4> host(cnt);
  for (size_t i = 0; i < cnt; i++) host[i] = make_float4(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], 0.0f);
  hipStream_t aux;
  if (int rc = aux_stream(c, &aux)) return rc;
  // a size change reallocates stream-ordered on the context's stream: a plain
  // hipFree would wait for every stream on the device
  if (c->d_lut && c->lut_n != n) {
    hipFreeAsync(c->d_lut, aux);
    c->d_lut = nullptr;
    if (c->d_lut_yuv) hipFreeAsync(c->d_lut_yuv, aux);
    c->d_lut_yuv = nullptr;
  }
  c->lut_yuv_scale = -1.0f;
  c->lut8x_ok = false;
  if (!c->d_lut) {
    hipError_t e = hipMallocAsync((void**)&c->d_lut, cnt * sizeof(float4), aux);
    if (e != hipSuccess) {
      c->d_lut = nullptr;
      return fail(c, H2S_E_OOM, "LUT device allocation failed");
    }
  }
  hipError_t e = table_copy(c, c->d_lut, host.data(), cnt * sizeof(float4));
  if (e != hipSuccess) return hip_fail(c, e, "LUT upload");
  c->lut_n = n;
  return 0;
}

int h2s_set_params(h2s_ctx* c, const h2s_params* p) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  if (!p) return fail(c, H2S_E_INVALID_ARG, "params is NULL");
  int rc = validate_params(c, p);
  if (rc) return rc;
  DeviceGuard g(c->device);
  if ((rc = drain_launches(c))) return rc;
  hipStream_t aux;
  if ((rc = aux_stream(c, &aux))) return rc;
  std::vector<uint16_t> eq;
  KParams k;
  resolve(p, &k, &eq);
  if (!c->d_eq) {
    hipError_t e = hipMalloc((void**)&c->d_eq, 4096 * sizeof(uint16_t));
    if (e != hipSuccess) {
      c->d_eq = nullptr;
      return fail(c, H2S_E_OOM, "eq table allocation failed");
    }
  }
  hipError_t e = table_copy(c, c->d_eq, eq.data(), eq.size() * sizeof(uint16_t));
  if (e != hipSuccess) return hip_fail(c, e, "eq table upload");
  {
    std::vector<float4> pq;
    // (x 10000/npl for either input transfer: the libplacebo branch's IPT form
    // decodes PQ L'M'S' through it for HLG input too)
    build_pq_table(10000.0 / p->npl, &pq);
    if (!c->d_pq && (e = hipMalloc((void**)&c->d_pq, pq.size() * sizeof(float4))) != hipSuccess) {
      c->d_pq = nullptr;
      return fail(c, H2S_E_OOM, "PQ table allocation failed");
    }
    if ((e = table_copy(c, c->d_pq, pq.data(), pq.size() * sizeof(float4))) != hipSuccess)
      return hip_fail(c, e, "PQ table upload");
    if (!c->d_pqi) {
      std::vector<float4> pqi;
      build_pqi_table(&pqi);
      if ((e = hipMalloc((void**)&c->d_pqi, pqi.size() * sizeof(float4))) != hipSuccess) {
        c->d_pqi = nullptr;
        return fail(c, H2S_E_OOM, "PQ encode table allocation failed");
      }
      if ((e = table_copy(c, c->d_pqi, pqi.data(), pqi.size() * sizeof(float4))) != hipSuccess)
        return hip_fail(c, e, "PQ encode table upload");
    }
    if (!c->d_hlg && p->transfer_in == H2S_TRC_HLG) {   // parameter-independent: built once
      std::vector<float4> hlg;
      build_hlg_table(&hlg);
      if ((e = hipMalloc((void**)&c->d_hlg, hlg.size() * sizeof(float4))) != hipSuccess) {
        c->d_hlg = nullptr;
        return fail(c, H2S_E_OOM, "HLG table allocation failed");
      }
      if ((e = table_copy(c, c->d_hlg, hlg.data(), hlg.size() * sizeof(float4))) != hipSuccess)
        return hip_fail(c, e, "HLG table upload");
    }
  }
  c->params = *p;
  c->k = k;
  c->params_set = true;
  h2s_peak_reset(c);  // a new parameter set starts a new sequence
  return 0;
}

// FastParams from the resolved KParams (same constants, scales folded)
static void resolve_fast(const h2s_ctx* c, const KParams& k, FastParams* F) {
  memset(F, 0, sizeof(*F));
  const h2s_params* p = &c->params;
  const int sh = p->bits_in - 8;
  const double ys = 1.0 / (219 << sh), yo = -(double)(16 << sh) / (219 << sh);
  const double cs = 1.0 / (224 << sh), co = -(double)(128 << sh) / (224 << sh);
  const double kr = 0.2627, kb = 0.0593, kg = 1.0 - kr - kb;
  const double mrcr = 2.0 * (1.0 - kr), mgcb = -2.0 * kb * (1.0 - kb) / kg, mgcr = -2.0 * kr * (1.0 - kr) / kg,
               mbcb = 2.0 * (1.0 - kb);
  F->ys = (float)ys;
  F->k_r = (float)(yo + mrcr * co);
  F->k_g = (float)(yo + (mgcb + mgcr) * co);
  F->k_b = (float)(yo + mbcb * co);
  F->y_off_c = (float)yo;
  F->c_mid = (float)(128 << sh);
  for (int odd = 0; odd < 2; odd++) {
    const double d = odd ? 8.0 : 4.0;
    F->a_rv[odd] = (float)(mrcr * cs / d);
    F->a_gu[odd] = (float)(mgcb * cs / d);
    F->a_gv[odd] = (float)(mgcr * cs / d);
    F->a_bu[odd] = (float)(mbcb * cs / d);
  }
  F->log2_lin_scale = (float)log2((p->transfer_in == H2S_TRC_HLG ? 1000.0 : 10000.0) / p->npl);
  F->log2_pq_scale = (float)log2(10000.0 / p->npl);
  {
    // k_tile takes a tile's steps without the exact-path ballot when every
    // pixel's E stays below the table's end: staged luma <= safe_y and
    // |centred chroma| <= safe_c (the legal half-range) give
    // E <= Y' + max_c sum |a| * safe_c < PQ_EMAX.  Table forms only (E staged
    // in segment units + 1); the direct HLG form has no exact path
    const bool table = p->transfer_in == H2S_TRC_PQ || k.pipe != h2s::PIPE_LIBPLACEBO;
    const double safe_c = (double)(112 << sh);
    const double amax = std::max(std::max(fabs(mrcr), fabs(mgcb) + fabs(mgcr)), fabs(mbcb)) * cs;
    const double ymax = (double)h2s::PQ_EMAX - amax * safe_c - 1e-3;
    F->safe_c = table ? (float)safe_c : HUGE_VALF;
    F->safe_y = table ? (float)(ymax * h2s::PQ_SEG + 1.0) : HUGE_VALF;
  }
  F->lr = k.lr, F->lg = k.lg, F->lb = k.lb, F->desat = k.desat;
  F->rein_p = k.rein_p, F->rein_k = k.rein_k;
  F->hable_peak_inv = k.hable_peak_inv;
  F->hable_ka = (float)(2.1 / 15.0 * (double)k.hable_peak_inv);
  F->hable_kb = (float)(0.25 / 15.0 * (double)k.hable_peak_inv);
  F->mob_j = k.mob_j, F->mob_a = k.mob_a, F->mob_b = k.mob_b, F->mob_k = k.mob_k;
  F->npl_1e4 = k.npl_1e4, F->e4_npl = k.e4_npl;
  F->b_e1min = (float)pq_encode_d(1e-6 * p->npl / 10000.0);
  F->tw_fold = (float)(p->npl / k.t_white);
  // libplacebo branch: 255 ((x ainv)^(1/2.4) - b) as exp2(log2(x)/2.4 + k1) - k2
  F->lp_k1 = (float)(log2((double)k.enc_ainv) / 2.4 + log2(255.0));
  F->lp_k2 = (float)(255.0 * (double)k.enc_b);
  F->lp_xmax = (float)(pow(1.0 + (double)k.enc_b, 2.4) / (double)k.enc_ainv * 1.001);
  F->nm1 = (float)(c->lut_n - 1);
  F->inv255 = 1.0f / 255.0f;
  F->qscale = k.qscale;
  F->c56 = 56.0f * k.qscale;
  for (int i = 0; i < 3; i++) F->k709[i] = k.k709[i], F->kcb[i] = k.kcb[i], F->kcr[i] = k.kcr[i];
  F->lp_ipt = k.lp_ipt;
  F->lp_qs_f = k.lp_qs / 255.0f;
  F->lp_qo = k.lp_qo;
  for (int i = 0; i < 3; i++) {
    F->lp_ky[i] = (float)((double)k.k709[i] / 255.0 * 219.0 * (double)k.qscale);
    F->lp_kcb[i] = (float)((double)k.kcb[i] / 255.0 * 56.0 * (double)k.qscale);
    F->lp_kcr[i] = (float)((double)k.kcr[i] / 255.0 * 56.0 * (double)k.qscale);
  }
  F->lp_cy = 16.0f * k.qscale + 0.5f;
  F->lp_dith = k.lp_dith;
  F->in_mask2 = k.in_mask | (k.in_mask << 16);
  for (int i = 0; i < 9; i++)
    F->ipt_r2l[i] = (float)(k.ipt_r2l[i] * k.ipt_npl), F->ipt_l2r[i] = (float)(k.ipt_l2r[i] * (p->npl / k.t_white));
  F->pqi_tab = c->d_pqi;
  F->lut_off = k.lut_enabled ? 0 : 1;
  F->n_nw = k.n_nw;
  F->tw_1e4 = (float)(k.t_white / 10000.0);
  for (int i = 0; i < 9; i++) F->m709[i] = k.m709[i];
  h2s::curve_fast(k, static_cast<h2s::CurveConsts*>(F));
  const int n = c->lut_n;
  F->log2_nm1 = (float)log2((double)(n - 1));
  F->s_max = nextafterf((float)(n - 1), 0.0f);
  F->x_max = 0.999999f;  // (N-1) * x_max^(1/2.4) stays > 3 ulp below N-1
  F->stride_g = (float)(12 * n);
  F->stride_b = (float)(12 * n * n);
  F->og = 12 * n;
  F->ob = 12 * n * n;
  F->c111 = 12 * (1 + n + n * n);
  F->cr = F->c111 - 12;
  F->cg = F->c111 - F->og;
  F->cb = F->c111 - F->ob;
  F->lut_yuv = c->d_lut_yuv;
  F->lut_bytes = 12 * n * n * n;
  F->lut8x = c->d_lut8x;
  F->eq_lut = c->d_eq;
  F->eq_n = k.qmax + 1;
  F->c_bias = 128.0f * k.qscale + 0.5f;
  F->shift_out = k.shift_out;
  F->rep_rs = k.expand_rep && k.shift_out ? 8 - k.shift_out : 31;
  F->dither = k.dither;
  F->out8 = p->bits_out == 8 ? 1 : 0;
  // the table k_tile stages for its input transfer: the PQ EOTF, or for HLG
  // input on the CPU chain the inverse OETF (the libplacebo branch keeps the
  // PQ table for its IPT form and evaluates the HLG curve directly)
  F->pq_tab = p->transfer_in == H2S_TRC_HLG && k.pipe != h2s::PIPE_LIBPLACEBO ? c->d_hlg : c->d_pq;
}

// the libplacebo branch's lut3d 8-bit table (k_build_lut8x): allocated on
// the context stream once, rebuilt on s after every h2s_set_lut
static int ensure_lut8x(h2s_ctx* c, hipStream_t s) {
  if (c->d_lut8x && c->lut8x_ok) return 0;
  if (!c->d_lut8x) {
    hipStream_t aux;
    if (int rc = aux_stream(c, &aux)) return rc;
    hipError_t e = hipMallocAsync((void**)&c->d_lut8x, sizeof(unsigned) << 24, aux);
    if (e == hipSuccess) e = hipStreamSynchronize(aux);
    if (e != hipSuccess) {
      c->d_lut8x = nullptr;
      return fail(c, H2S_E_OOM, "lut3d 8-bit table allocation failed");
    }
  }
  hipError_t e = h2s::build_lut8x(c->d_lut, c->lut_n, c->d_lut8x, s);
  if (e != hipSuccess) return hip_fail(c, e, "lut3d 8-bit table build");
  c->lut8x_ok = true;
  return 0;
}

static int ensure_lut_yuv(h2s_ctx* c, const KParams& k, hipStream_t s) {
  if (k.rgba8) return ensure_lut8x(c, s);   // the libplacebo branch reads only its 8-bit table
  if (c->d_lut_yuv && c->lut_yuv_scale == k.qscale && c->lut_yuv_rgb == k.rgba8) return 0;
  const size_t cnt = (size_t)c->lut_n * c->lut_n * c->lut_n;
  if (!c->d_lut_yuv) {  // beside d_lut: stream-ordered on the context stream, complete before s uses it
    hipStream_t aux;
    if (int rc = aux_stream(c, &aux)) return rc;
    // zero-filled tail: a coordinate clamped to exactly N-1 (k_tile's
    // H2S_EXPCLAMP form) names cell N-1, whose corners past the lattice edge
    // carry weight 0 but are still read; the scalar-record steps read them
    // without the buffer resource's bounds check, so they must be mapped
    const size_t pad = 12 * (1 + (size_t)c->lut_n + (size_t)c->lut_n * c->lut_n) + 16;
    hipError_t e = hipMallocAsync((void**)&c->d_lut_yuv, cnt * 3 * sizeof(float) + pad, aux);
    if (e == hipSuccess) e = hipMemsetAsync((uint8_t*)c->d_lut_yuv + cnt * 3 * sizeof(float), 0, pad, aux);
    if (e == hipSuccess) e = hipStreamSynchronize(aux);
    if (e != hipSuccess) {
      c->d_lut_yuv = nullptr;
      return fail(c, H2S_E_OOM, "YUV lattice allocation failed");
    }
  }
  h2s::YuvLutConsts K;
  K.s = k.qscale;
  K.rgb = k.rgba8;
  for (int i = 0; i < 3; i++) K.k709[i] = k.k709[i], K.kcb[i] = k.kcb[i], K.kcr[i] = k.kcr[i];
  hipError_t e = h2s::build_lut_yuv(c->d_lut, c->d_lut_yuv, c->lut_n, K, s);
  if (e != hipSuccess) return hip_fail(c, e, "YUV lattice build");
  c->lut_yuv_scale = k.qscale;
  c->lut_yuv_rgb = k.rgba8;
  return 0;
}

static int prepare(h2s_ctx* c, KParams* k, bool need_lut = true) {
  if (!c->params_set) return fail(c, H2S_E_INVALID_ARG, "h2s_set_params was not called");
  if (need_lut && c->params.lut_enabled && !c->d_lut)
    return fail(c, H2S_E_LUT_MISSING, "lut_enabled but no LUT loaded (h2s_set_lut)");
  *k = c->k;
  k->lut = c->d_lut;
  k->lut_n = c->lut_n;
  k->lut_sg = c->lut_n;
  k->lut_sb = c->lut_n * c->lut_n;
  k->lut_max = (float)(c->lut_n - 1);
  k->eq_lut = c->d_eq;
  return 0;
}

// the generic kernel over the columns right of the last whole 64-pixel tile
// (left-sited chroma needs no left neighbour, so the seam is exact)
static hipError_t launch_tail(const KParams& k, int nframes, bool vec, bool out8, hipStream_t s, int tw) {
  const int w64 = k.W & ~(tw - 1);
  KParams kt = k;
  kt.gx0 = w64 / 8;
  kt.ngx = (k.cw - w64 / 2 + 3) / 4;
  kt.total = (long long)nframes * k.ch * kt.ngx;
  return h2s::launch_process(kt, vec, out8, s);
}

// BICUBIC chroma taps (oracle_chroma_taps): horizontal 7 taps around the
// left-sited position, vertical 8 around the centre-sited one, normalised
static void chroma_taps(float* wx7, float* wy8) {
  auto bic = [](double x) {
    const double B = 0.0, C = 0.6;
    x = fabs(x);
    if (x < 1.0) return ((12 - 9 * B - 6 * C) * x * x * x + (-18 + 12 * B + 6 * C) * x * x + (6 - 2 * B)) / 6.0;
    if (x < 2.0) return ((-B - 6 * C) * x * x * x + (6 * B + 30 * C) * x * x + (-12 * B - 48 * C) * x + (8 * B + 24 * C)) / 6.0;
    return 0.0;
  };
  double tx[7], ty[8], sx = 0, sy = 0;
  for (int i = 0; i < 7; i++) sx += (tx[i] = bic((i - 3) / 2.0));
  for (int j = 0; j < 8; j++) sy += (ty[j] = bic((j - 3.5) / 2.0));
  for (int i = 0; i < 7; i++) wx7[i] = (float)(tx[i] / sx);
  for (int j = 0; j < 8; j++) wy8[j] = (float)(ty[j] / sy);
}

// BICUBIC chroma: frame by frame, per-pixel chroma into the context scratch
// then the decimation (h2s_kernels.hip launch_two_pass)
static hipError_t launch_two_pass_frames(const h2s_ctx* c, const KParams& k, bool out8, int nframes, hipStream_t s) {
  float wx[7], wy[8];
  chroma_taps(wx, wy);
  for (int f = 0; f < nframes; f++) {
    KParams kf = k;
    for (int p = 0; p < 3; p++) {
      kf.in[p] += f * kf.in_fp[p];
      kf.out[p] += f * kf.out_fp[p];
    }
    kf.nframes = 1;
    kf.total = (long long)kf.ch * kf.ngx;
    kf.chr444 = c->d_chr;
    hipError_t e = h2s::launch_process_c444(kf, out8, s);
    if (e == hipSuccess) e = h2s::launch_chroma_bicubic(kf, wx, wy, out8, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

static hipError_t launch_chain(const h2s_ctx* c, const KParams& k, bool fast, bool vec, bool out8, int nframes,
                               hipStream_t s, const h2s::CurveConsts* cvf, bool tail, int dbg, float* dbg_out,
                               float2* chr444);

// BICUBIC chroma with the tile kernel, frame by frame: k_tile writes luma
// and every pixel's (Cb, Cr) into the context scratch (the generic C444
// kernel covers the width % 64 columns), then the decimation pass
static hipError_t launch_tile_two_pass(const h2s_ctx* c, const KParams& k, bool out8, int nframes, hipStream_t s) {
  float wx[7], wy[8];
  chroma_taps(wx, wy);
  for (int f = 0; f < nframes; f++) {
    KParams kf = k;
    for (int p = 0; p < 3; p++) {
      kf.in[p] += f * kf.in_fp[p];
      kf.out[p] += f * kf.out_fp[p];
    }
    kf.nframes = 1;
    kf.total = (long long)kf.ch * kf.ngx;
    kf.chr444 = c->d_chr;
    hipError_t e = launch_chain(c, kf, true, false, out8, 1, s, nullptr, false, 0, nullptr, c->d_chr);
    const int w64 = k.W & ~(h2s::TBW - 1);
    if (e == hipSuccess && w64 != k.W) {
      KParams kt = kf;
      kt.gx0 = w64 / 8;
      kt.ngx = (k.cw - w64 / 2 + 3) / 4;
      kt.total = (long long)k.ch * kt.ngx;
      e = h2s::launch_process_c444(kt, out8, s);
    }
    if (e == hipSuccess) e = h2s::launch_chroma_bicubic(kf, wx, wy, out8, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// one launch of the chain over nframes frames described by k.  cvf: per-frame
// curve records (dynamic peak, fast kernel); tail = false leaves the ragged
// right columns to the caller; dbg > 0: the tile kernel's debug instance for
// that stage, writing frame 0's planes to dbg_out
static hipError_t launch_chain(const h2s_ctx* c, const KParams& k, bool fast, bool vec, bool out8, int nframes,
                               hipStream_t s, const h2s::CurveConsts* cvf = nullptr, bool tail = true, int dbg = 0,
                               float* dbg_out = nullptr, float2* chr444 = nullptr) {
  if (!fast) {
    if (c->params.chroma_filter == H2S_CHROMA_BICUBIC) return launch_two_pass_frames(c, k, out8, nframes, s);
    return h2s::launch_process(k, vec, out8, s);
  }
  if (c->params.chroma_filter == H2S_CHROMA_BICUBIC && !dbg && !chr444) return launch_tile_two_pass(c, k, out8, nframes, s);
  FastParams F;
  resolve_fast(c, k, &F);
  for (int p = 0; p < 3; p++) {
    F.in[p] = k.in[p], F.in_ls[p] = k.in_ls[p], F.in_fp[p] = k.in_fp[p];
    F.out[p] = k.out[p], F.out_ls[p] = k.out_ls[p], F.out_fp[p] = k.out_fp[p];
  }
  // k_tile covers the whole 64-pixel tiles; the chroma right halo of its last
  // tile reads the real column (F.cw stays the frame's), so the split is exact
  const int tw = h2s::TBW;
  const int w64 = k.W & ~(tw - 1);
  F.W = w64, F.H = k.H, F.cw = k.cw, F.ch = k.ch;
  F.chroma_edge = k.chroma_edge;
  for (int p = 0; p < 3; p++) {
    const long long ib = (long long)(p ? k.ch : k.H) * k.in_ls[p], ob = (long long)(p ? k.ch : k.H) * k.out_ls[p];
    F.in_bytes[p] = (int)(ib < 0x7fffffff ? ib : 0x7fffffff);
    F.out_bytes[p] = (int)(ob < 0x7fffffff ? ob : 0x7fffffff);
  }
  F.nbx = (unsigned)(w64 / tw);
  F.nby = (unsigned)((k.H + h2s::TBH - 1) / h2s::TBH);
  F.nframes = (unsigned)nframes;
  F.tpb = c->tiles_per_block;
  F.cv_frames = cvf;
  F.dbg = dbg_out;
  F.dbg_w = k.W;
  F.dbg_lut = c->d_lut;
  F.inv_nm1 = 1.0f / (float)(c->lut_n - 1);
  F.chr444 = chr444;
  F.chr_w = k.W;
  F.inv_c56 = 1.0f / F.c56;
  const int desat = !k.desat_on ? 0 : (k.lr == 1.0f && k.lg == 1.0f && k.lb == 1.0f ? 2 : 1);
  hipError_t e = h2s::launch_fast(F, k.transfer, k.tonemap, desat, k.pipe == h2s::PIPE_LIBPLACEBO ? 1 : 0, s, dbg);
  if (e != hipSuccess || w64 == k.W || !tail || dbg) return e;
  return launch_tail(k, nframes, vec, out8, s, tw);
}

// the tile kernel serves: both of the reference's chains (the CPU chain, and
// the libplacebo branch with the LUT on: k_tile<..., LP = 1>), the LUT on at
// N <= 177 (its lattice byte offsets are formed in float32, exact for
// multiples of 4 below 2^26 = 12 * 177^3 + margin), the default [EXT]
// switches, 10/12-bit input and BASELINE's operators; frames with a 64-wide
// tile and 16-byte aligned rows
static bool fast_params_ok(const h2s_ctx* c, const KParams& k) {
  const h2s_params& p = c->params;
  if (!c->fast_enabled || !h2s::fast_supported(k.tonemap)) return false;
  if (c->lp_exact && k.pipe == h2s::PIPE_LIBPLACEBO) return false;
  // the LUT off runs on the tile kernel for the libplacebo branch only (the
  // CPU chain's legacy closed form stays on the generic kernel)
  if (!k.lut_enabled && k.pipe != h2s::PIPE_LIBPLACEBO) return false;
  // the CPU chain forms lattice byte offsets in float32 (exact to N = 177);
  // the libplacebo branch reads its 8-bit table, any N
  if (k.lut_enabled && c->lut_n > 177 && !k.rgba8) return false;
  if (k.lut_in16) return false;
  // BICUBIC: the tile kernel runs pass 1 frame by frame (not under dynamic peak detection)
  if (p.chroma_filter == H2S_CHROMA_BICUBIC && p.peak_detect) return false;
  return true;
}

static int choose_path(const h2s_ctx* c, const KParams& k, const h2s_frames* din, const h2s_frames* dout,
                       bool out8) {
  const int tw = h2s::TBW;
  if (fast_params_ok(c, k) && tile_ok(din, dout, out8, tw))
    return (din->width & (tw - 1)) ? H2S_PATH_TILE_TAIL : H2S_PATH_TILE;
  return c->params.chroma_filter == H2S_CHROMA_BICUBIC ? H2S_PATH_TWO_PASS : H2S_PATH_GENERIC;
}

static int ensure_chr(h2s_ctx* c, const KParams& k) {
  // whole 32-row tiles: k_tile writes the rows of its bottom tile past H
  const size_t need = (size_t)k.W * (size_t)((k.H + h2s::TBH - 1) / h2s::TBH * h2s::TBH);
  if (need <= c->chr_cap) return 0;
  if (c->d_chr) hipFree(c->d_chr);
  c->d_chr = nullptr;
  c->chr_cap = 0;
  if (hipMalloc((void**)&c->d_chr, need * sizeof(float2)) != hipSuccess) {
    c->d_chr = nullptr;
    return fail(c, H2S_E_OOM, "bicubic chroma scratch allocation failed");
  }
  c->chr_cap = need;
  return 0;
}

// libplacebo-style detected peak (PARITY UNPINNED; model in DESIGN.md §4.6),
// all on the device (h2s_peak.h): k_peak_stats* (per-block partials and the
// percentile histograms) -> k_peak_frame (per-frame statistic) ->
// k_peak_curves (the IIR in frame order from the context's device state, and
// one curve record per frame) -> the conversion, which reads the records.
// h2s_process queues all of it on the caller's stream and returns; the state
// comes back to the host only on demand (h2s_peak_state).
static h2s::PeakModel peak_model(const h2s_ctx* c, const KParams& k) {
  h2s::PeakModel m;
  m.t_white = k.t_white, m.t_black = k.t_black, m.knee_off = k.knee_off;
  m.contrast = k.sp_contrast, m.tm_param = c->params.tm_param, m.static_peak = k.peak;
  m.smoothing = k.pd_smoothing, m.scene_low = k.pd_scene_low, m.scene_high = k.pd_scene_high;
  m.percentile = k.pd_percentile, m.min_peak = k.pd_min;
  m.iir_a = k.pd_smoothing > 0.0 ? 1.0 - exp(-1.0 / k.pd_smoothing) : 1.0;
  m.npx = (double)k.W * k.H;
  m.nblocks = c->peak_blocks;
  m.pct = k.pd_percentile < 100.0 ? 1 : 0;
  m.family = k.tonemap;
  m.pq = h2s::pq_refs(k.t_white, k.t_black);
  return m;
}

// device buffer of at least `need` bytes (grown, never shrunk); a grown
// buffer is freed only after the launches that read the old one (hipFree
// synchronises)
static int ensure_dev(h2s_ctx* c, void** buf, size_t* cap, size_t need, const char* what) {
  if (need <= *cap) return 0;
  if (*buf) hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  if (hipMalloc(buf, need) != hipSuccess) {
    *buf = nullptr;
    return fail(c, H2S_E_OOM, std::string(what) + " allocation failed");
  }
  *cap = need;
  return 0;
}

static int ensure_peak_state(h2s_ctx* c) {
  if (c->d_pk) return 0;
  if (hipMalloc((void**)&c->d_pk, 2 * sizeof(h2s::PeakState)) != hipSuccess) {
    c->d_pk = nullptr;
    return fail(c, H2S_E_OOM, "peak state allocation failed");
  }
  hipStream_t aux;
  if (int rc = aux_stream(c, &aux)) return rc;
  hipError_t e = hipMemsetAsync(c->d_pk, 0, 2 * sizeof(h2s::PeakState), aux);
  if (e == hipSuccess) e = hipStreamSynchronize(aux);
  return e == hipSuccess ? 0 : hip_fail(c, e, "peak state reset");
}

// the statistics, the curves and the state are one context's scratch: a call
// on another stream waits (on the device) for the previous call's use of
// them, so consecutive calls see the state in call order
static int peak_order(h2s_ctx* c, hipStream_t s) {
  if (!c->peak_ev) {
    hipError_t e = hipEventCreateWithFlags(&c->peak_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      c->peak_ev = nullptr;
      return hip_fail(c, e, "peak event");
    }
  }
  if (!c->peak_pending) return 0;
  hipError_t e = hipStreamWaitEvent(s, c->peak_ev, 0);
  return e == hipSuccess ? 0 : hip_fail(c, e, "peak ordering");
}

static int peak_done(h2s_ctx* c, hipStream_t s) {
  hipError_t e = hipEventRecord(c->peak_ev, s);
  if (e != hipSuccess) return hip_fail(c, e, "peak event");
  c->peak_pending = true;
  return 0;
}

// per-frame statistic (PQ peak measurement, average PQ) of the batch k binds
// into c->d_fstat, queued on s as two launches (k_peak_stats*, then
// k_peak_finish: one block per frame folds its records; the last one, st set,
// runs the IIR from *st and writes the curve records to out).  d_stats holds,
// for stats_nf frames: partial records | histograms | the finish counter; the
// histograms and the counter are zero between launches (cleared at
// allocation, left zero by the kernels)
static int frame_stats(h2s_ctx* c, const KParams& k, int nframes, hipStream_t s, h2s::PeakState* st,
                       h2s::CurveConsts* out, int f0 = 0) {
  const h2s::PeakModel m = peak_model(c, k);
  if (nframes > c->stats_nf) {
    const size_t nf = (size_t)nframes;
    const size_t part = nf * h2s::PEAK_BLOCKS_MAX * sizeof(float2), zero = (nf * h2s::PEAK_BINS + 1) * sizeof(unsigned);
    if (c->d_stats) hipFree(c->d_stats);
    c->d_stats = nullptr;
    c->stats_nf = 0;
    if (hipMalloc(&c->d_stats, part + zero) != hipSuccess) {
      c->d_stats = nullptr;
      return fail(c, H2S_E_OOM, "peak statistics allocation failed");
    }
    hipError_t e = hipMemsetAsync(static_cast<char*>(c->d_stats) + part, 0, zero, s);
    if (e != hipSuccess) return hip_fail(c, e, "peak statistics clear");
    c->stats_nf = nframes;
  }
  if (int rc = ensure_dev(c, (void**)&c->d_fstat, &c->fstat_cap, (size_t)(f0 + nframes) * sizeof(double2),
                         "peak statistics"))
    return rc;
  const size_t nf = (size_t)c->stats_nf;
  float2* d_part = static_cast<float2*>(c->d_stats);
  h2s::PeakTail T;
  T.M = m;
  T.fstat = c->d_fstat + f0;
  T.hist = reinterpret_cast<unsigned*>(d_part + nf * h2s::PEAK_BLOCKS_MAX);
  T.done = T.hist + nf * h2s::PEAK_BINS;
  T.st = st;
  T.out = out;
  T.nframes = nframes;
  T.form = c->peak_form;
  hipError_t e = h2s::launch_peak_stats(k, d_part, T, s);
  return e == hipSuccess ? 0 : hip_fail(c, e, "peak statistics");
}

// k restricted to frames [f0, f0 + n)
static KParams frame_range(const KParams& k, int f0, int n) {
  KParams kf = k;
  for (int p = 0; p < 3; p++) {
    kf.in[p] += (long long)f0 * kf.in_fp[p];
    kf.out[p] += (long long)f0 * kf.out_fp[p];
  }
  kf.nframes = n;
  kf.total = (long long)n * kf.ch * kf.ngx;
  return kf;
}

static int peak_streams(h2s_ctx* c, int nev) {
  for (hipStream_t& ps : c->pk_s)
    if (!ps) {
      hipError_t e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
      if (e != hipSuccess) {
        ps = nullptr;
        return hip_fail(c, e, "peak stream");
      }
    }
  while ((int)c->pk_ev.size() < nev) {
    hipEvent_t ev;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "peak event");
    c->pk_ev.push_back(ev);
  }
  return 0;
}

// The pipelined schedule (tile kernel, whole tiles): the statistics of chunk
// j + 1 run on their own stream while chunk j converts, and consecutive
// chunks convert on alternating streams, so that neither a chunk boundary
// nor the statistics leave the chip idle.  The state still advances frame by
// frame in order (the statistics stream is serial), exactly as one launch.
static int run_dynamic_peak_chunked(h2s_ctx* c, const KParams& k, bool vec, bool out8, int nframes, hipStream_t s) {
  const int C = c->peak_chunk, nch = (nframes + C - 1) / C;
  int rc;
  // every allocation before the first launch (hipFree of a grown buffer
  // would wait for the device)
  if ((rc = peak_streams(c, nch + 2)) ||
      (rc = ensure_dev(c, (void**)&c->d_fstat, &c->fstat_cap, (size_t)nframes * sizeof(double2), "peak statistics")))
    return rc;
  hipStream_t ss = c->pk_s[0], st[2] = {s, c->pk_s[1]};
  hipEvent_t ev_start = c->pk_ev[0], ev_end = c->pk_ev[1];
  hipError_t e = hipEventRecord(ev_start, s);
  if (e == hipSuccess) e = hipStreamWaitEvent(ss, ev_start, 0);
  if (e == hipSuccess) e = hipStreamWaitEvent(st[1], ev_start, 0);
  if (e != hipSuccess) return hip_fail(c, e, "peak schedule");
  // an error exit still joins what was queued on the two internal streams
  // into s (best effort), so the caller's stream (and queued_exit's launch
  // event) covers all of it
  auto fail_joined = [&](int code) {
    if (hipEventRecord(ev_end, st[1]) == hipSuccess) (void)hipStreamWaitEvent(s, ev_end, 0);
    if (hipEventRecord(ev_start, ss) == hipSuccess) (void)hipStreamWaitEvent(s, ev_start, 0);
    return code;
  };
  for (int j = 0; j < nch; j++) {
    const int f0 = j * C, n = std::min(C, nframes - f0);
    const KParams kj = frame_range(k, f0, n);
    if ((rc = frame_stats(c, kj, n, ss, c->d_pk, c->d_curve + f0, f0))) return fail_joined(rc);
    hipEvent_t ev = c->pk_ev[2 + j];
    if ((e = hipEventRecord(ev, ss)) != hipSuccess || (e = hipStreamWaitEvent(st[j & 1], ev, 0)) != hipSuccess)
      return fail_joined(hip_fail(c, e, "peak schedule"));
    if ((e = launch_chain(c, kj, true, vec, out8, n, st[j & 1], c->d_curve + f0, false)) != hipSuccess)
      return fail_joined(hip_fail(c, e, "kernel launch"));
  }
  // s joins the statistics stream (the state) and the second conversion stream
  if ((e = hipEventRecord(ev_end, st[1])) != hipSuccess || (e = hipStreamWaitEvent(s, ev_end, 0)) != hipSuccess ||
      (e = hipStreamWaitEvent(s, c->pk_ev[2 + nch - 1], 0)) != hipSuccess)
    return fail_joined(hip_fail(c, e, "peak schedule"));
  return peak_done(c, s);
}

// statistics, then the frames in order, each with the BT.2390 / spline
// constants of its smoothed peak.  The fast kernel takes every frame's curve
// in one launch (a record per frame, selected by the tile's frame index), so
// the chip stays full; the generic kernel and the ragged tail columns go frame
// by frame, each launch reading its frame's record.
static int run_dynamic_peak(h2s_ctx* c, const KParams& k, bool fast, bool vec, bool out8, int nframes, hipStream_t s) {
  int rc;
  if ((rc = ensure_peak_state(c)) || (rc = peak_order(c, s))) return rc;
  if ((rc = ensure_dev(c, (void**)&c->d_curve, &c->curve_cap, (size_t)nframes * sizeof(h2s::CurveConsts), "curve records")))
    return rc;
  if (fast && (k.W & (h2s::TBW - 1)) == 0 && c->peak_chunk > 0 && nframes > c->peak_chunk)
    return run_dynamic_peak_chunked(c, k, vec, out8, nframes, s);
  if ((rc = frame_stats(c, k, nframes, s, c->d_pk, c->d_curve))) return rc;
  hipError_t e;
  if (fast) {
    e = launch_chain(c, k, true, vec, out8, nframes, s, c->d_curve, false);
    if (e != hipSuccess) return hip_fail(c, e, "kernel launch");
  }
  if (!fast || (k.W & (h2s::TBW - 1)) != 0) {
    for (int f = 0; f < nframes; f++) {
      KParams kf = frame_range(k, f, 1);
      kf.cv = c->d_curve + f;
      e = fast ? launch_tail(kf, 1, vec, out8, s, h2s::TBW) : launch_chain(c, kf, false, vec, out8, 1, s);
      if (e != hipSuccess) return hip_fail(c, e, "kernel launch");
    }
  }
  return peak_done(c, s);
}

// the host-side peak calls act on the state as the context's queued work
// leaves it: they wait for that work first (its launch events and the last
// peak launch), then run on the context stream and wait for it
static int peak_sync(h2s_ctx* c, hipStream_t* aux) {
  int rc;
  if ((rc = drain_launches(c)) || (rc = ensure_peak_state(c)) || (rc = aux_stream(c, aux))) return rc;
  if (c->peak_pending) {
    hipError_t e = hipEventSynchronize(c->peak_ev);
    if (e != hipSuccess) return hip_fail(c, e, "peak launches");
    c->peak_pending = false;
  }
  return 0;
}

int h2s_peak_reset(h2s_ctx* c) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  DeviceGuard g(c->device);
  hipStream_t aux;
  if (int rc = peak_sync(c, &aux)) return rc;
  hipError_t e = hipMemsetAsync(c->d_pk, 0, sizeof(h2s::PeakState), aux);
  if (e == hipSuccess) e = hipStreamSynchronize(aux);
  return e == hipSuccess ? 0 : hip_fail(c, e, "peak state reset");
}

int h2s_peak_feed(h2s_ctx* c, const double* fmax, const double* favg, int n) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  if (n < 0 || (n > 0 && (!fmax || !favg))) return fail(c, H2S_E_INVALID_ARG, "bad statistics arrays");
  KParams k;
  int rc = prepare(c, &k, false);  // the statistics need no LUT
  if (rc) return rc;
  if (n == 0) return 0;
  DeviceGuard g(c->device);
  hipStream_t aux;
  if ((rc = peak_sync(c, &aux))) return rc;
  if ((rc = ensure_dev(c, (void**)&c->d_fstat, &c->fstat_cap, (size_t)n * sizeof(double2), "peak statistics"))) return rc;
  std::vector<double2> st(n);
  for (int i = 0; i < n; i++) st[i] = make_double2(fmax[i], favg[i]);
  // the same device IIR as h2s_process (bit-identical state either way)
  hipError_t e = hipMemcpyAsync(c->d_fstat, st.data(), n * sizeof(double2), hipMemcpyHostToDevice, aux);
  if (e == hipSuccess) e = h2s::launch_peak_curves(c->d_fstat, n, peak_model(c, k), c->d_pk, nullptr, aux);
  if (e == hipSuccess) e = hipStreamSynchronize(aux);
  return e == hipSuccess ? 0 : hip_fail(c, e, "peak feed");
}

int h2s_peak_state(const h2s_ctx* cc, double* max_pq, double* avg_pq, double* peak, int64_t* frames) {
  if (!cc) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  // logically const: waits for the context's queued work, copies the state back
  h2s_ctx* c = const_cast<h2s_ctx*>(cc);
  DeviceGuard g(c->device);
  hipStream_t aux;
  if (int rc = peak_sync(c, &aux)) return rc;
  h2s::PeakState st;
  hipError_t e = hipMemcpyAsync(&st, c->d_pk, sizeof(st), hipMemcpyDeviceToHost, aux);
  if (e == hipSuccess) e = hipStreamSynchronize(aux);
  if (e != hipSuccess) return hip_fail(c, e, "peak state read-back");
  if (max_pq) *max_pq = st.max;
  if (avg_pq) *avg_pq = st.avg;
  if (peak) *peak = st.peak;
  if (frames) *frames = st.frames;
  return 0;
}

int h2s_peak_stats(h2s_ctx* c, const h2s_frames* in, int nframes, double* fmax, double* favg, void* hip_stream) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  if (nframes < 0 || (nframes > 0 && (!fmax || !favg))) return fail(c, H2S_E_INVALID_ARG, "bad statistics arrays");
  KParams k;
  int rc = prepare(c, &k, false);  // the statistics need no LUT
  if (rc) return rc;
  if ((rc = check_frames(c, in, c->params.bits_in, "input"))) return rc;
  if (in->location != H2S_LOC_DEVICE) return fail(c, H2S_E_INVALID_ARG, "h2s_peak_stats takes device frames");
  if (nframes == 0) return 0;
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)hip_stream;
  h2s_frames out = *in;                       // geometry only: the statistics read the input planes
  fill_geometry(&k, in, &out, nframes);
  if ((rc = peak_order(c, s)) || (rc = frame_stats(c, k, nframes, s, nullptr, nullptr))) return rc;
  std::vector<double2> st(nframes);
  hipError_t e = hipMemcpyAsync(st.data(), c->d_fstat, nframes * sizeof(double2), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(c, e, "peak statistics read-back");
  for (int f = 0; f < nframes; f++) fmax[f] = st[f].x, favg[f] = st[f].y;
  return 0;
}

// frames [start, ...) of a batch
static h2s_frames frames_at(const h2s_frames* f, int start) {
  h2s_frames t = *f;
  for (int p = 0; p < 3; p++) t.data[p] = (uint8_t*)f->data[p] + (long long)start * f->frame_pitch[p];
  return t;
}

// Host frames in and/or out: the batch is cut into up to kMaxChunks chunks of
// whole frames; chunk i's H2D copy, kernel and D2H copy run on three streams
// so that copies of neighbouring chunks overlap the kernel and each other.
// Staging holds the whole batch (no buffer reuse, so no WAR hazards); all
// three streams start after the work already queued on `s`, and `s` waits
// for them before the call returns. din/dout: staged (or caller's device)
// descriptors for frame 0.
static int process_pipelined(h2s_ctx* c, KParams k, const h2s_frames* in, const h2s_frames* out,
                             const h2s_frames& din, const h2s_frames& dout, int nframes, bool fast, bool vec,
                             bool out8, hipStream_t s, bool dyn_peak) {
  const bool host_in = in->location == H2S_LOC_HOST, host_out = out->location == H2S_LOC_HOST;
  for (hipStream_t& ps : c->ps)
    if (!ps) {
      hipError_t e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
      if (e != hipSuccess) {
        ps = nullptr;
        return hip_fail(c, e, "pipeline stream");
      }
    }
  for (hipEvent_t& ev : c->pev)
    if (!ev) {
      hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      if (e != hipSuccess) {
        ev = nullptr;
        return hip_fail(c, e, "pipeline event");
      }
    }
  hipStream_t s_in = c->ps[0], s_cmp = c->ps[1], s_out = c->ps[2];
  const int per = (nframes + kMaxChunks - 1) / kMaxChunks, nch = (nframes + per - 1) / per;
  hipEvent_t ev_start = c->pev[2 * kMaxChunks], ev_done = c->pev[2 * kMaxChunks + 1];
  hipError_t e = hipEventRecord(ev_start, s);
  for (hipStream_t ps : c->ps)
    if (e == hipSuccess) e = hipStreamWaitEvent(ps, ev_start, 0);
  if (e != hipSuccess) return hip_fail(c, e, "pipeline ordering");
  const int slot = (int)(c->ev_count % kEvRing);
  const char* what = nullptr;
  for (int i = 0; i < nch && !what; i++) {
    const int f0 = i * per, nf = nframes - f0 < per ? nframes - f0 : per;
    const h2s_frames ci = frames_at(&din, f0), co = frames_at(&dout, f0);
    if (host_in) {
      const h2s_frames hi = frames_at(in, f0);
      if ((e = copy_frames(&ci, &hi, nf, s_in)) != hipSuccess) what = "host->device copy";
      else if ((e = hipEventRecord(c->pev[i], s_in)) != hipSuccess) what = "pipeline event";
      else if ((e = hipStreamWaitEvent(s_cmp, c->pev[i], 0)) != hipSuccess) what = "pipeline ordering";
      if (what) break;
    }
    if (c->timing && i == 0) {
      if (!c->ev0[slot]) {
        hipEventCreate(&c->ev0[slot]);
        hipEventCreate(&c->ev1[slot]);
      }
      hipEventRecord(c->ev0[slot], s_cmp);
    }
    fill_geometry(&k, &ci, &co, nf);
    if (dyn_peak) {
      if (int rc = run_dynamic_peak(c, k, fast, vec, out8, nf, s_cmp)) {
        for (hipStream_t ps : c->ps) hipStreamSynchronize(ps);
        return rc;
      }
    } else if ((e = launch_chain(c, k, fast, vec, out8, nf, s_cmp)) != hipSuccess) {
      what = "kernel launch";
    }
    if (!what && host_out) {
      const h2s_frames ho = frames_at(out, f0);
      if ((e = hipEventRecord(c->pev[kMaxChunks + i], s_cmp)) != hipSuccess) what = "pipeline event";
      else if ((e = hipStreamWaitEvent(s_out, c->pev[kMaxChunks + i], 0)) != hipSuccess) what = "pipeline ordering";
      else if ((e = copy_frames(&ho, &co, nf, s_out)) != hipSuccess) what = "device->host copy";
    }
  }
  if (what) {  // drain whatever was queued before returning the caller's buffers
    for (hipStream_t ps : c->ps) hipStreamSynchronize(ps);
    return hip_fail(c, e, what);
  }
  if (c->timing) {
    hipEventRecord(c->ev1[slot], s_cmp);
    c->ev_count++;
  }
  // s waits for the last stream of the chain (D2H if any, else compute)
  if ((e = hipEventRecord(ev_done, host_out ? s_out : s_cmp)) == hipSuccess) e = hipStreamWaitEvent(s, ev_done, 0);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    for (hipStream_t ps : c->ps) hipStreamSynchronize(ps);
    return hip_fail(c, e, "stream synchronize");
  }
  return 0;
}

int h2s_process(h2s_ctx* c, const h2s_frames* in, const h2s_frames* out, int nframes, void* hip_stream) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  if (nframes < 0) return fail(c, H2S_E_INVALID_ARG, "nframes < 0");
  KParams k;
  int rc = prepare(c, &k);
  if (rc) return rc;
  if ((rc = check_frames(c, in, c->params.bits_in, "input"))) return rc;
  if ((rc = check_frames(c, out, c->params.bits_out, "output"))) return rc;
  if (in->width != out->width || in->height != out->height)
    return fail(c, H2S_E_INVALID_ARG, "input and output frame sizes differ");
  if (nframes == 0) return 0;
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)hip_stream;
  const bool out8 = c->params.bits_out == 8;

  h2s_frames din = *in, dout = *out;
  const bool host_in = in->location == H2S_LOC_HOST, host_out = out->location == H2S_LOC_HOST;
  if (host_in || host_out) {
    const size_t ib = host_in ? frame_bytes(in) * nframes : 0, ob = host_out ? frame_bytes(out) * nframes : 0;
    const size_t need = ((ib + 255) / 256) * 256 + ob;
    if (need > c->stage_bytes) {
      if (c->d_stage) hipFree(c->d_stage);
      c->d_stage = nullptr;
      c->stage_bytes = 0;
      hipError_t e = hipMalloc(&c->d_stage, need);
      if (e != hipSuccess) {
        c->d_stage = nullptr;
        return fail(c, H2S_E_OOM, "staging allocation failed");
      }
      c->stage_bytes = need;
    }
    if (host_in) din = tight(in, c->d_stage);
    if (host_out) dout = tight(out, (uint8_t*)c->d_stage + ((ib + 255) / 256) * 256);
  }
  fill_geometry(&k, &din, &dout, nframes);
  const bool vec = vec_ok(&din, false) && vec_ok(&dout, out8);
  // fast path: the tile kernel over whole 64 x 32 tiles; the generic kernel
  // covers the rest (choose_path / fast_params_ok) and the ragged columns
  const int path = choose_path(c, k, &din, &dout, out8);
  const bool fast = path == H2S_PATH_TILE || path == H2S_PATH_TILE_TAIL;
  if (fast && k.lut_enabled && (rc = ensure_lut_yuv(c, k, s))) return rc;
  // BICUBIC chroma (generic two-pass, or k_tile pass 1) uses the context scratch
  const bool two_pass = c->params.chroma_filter == H2S_CHROMA_BICUBIC;
  if (two_pass) {
    if ((rc = ensure_chr(c, k))) return rc;
    // one context scratch (d_chr) for every two-pass launch: a launch on
    // another stream waits until the previous one has finished with it
    if (!c->chr_ev) {
      hipError_t e = hipEventCreateWithFlags(&c->chr_ev, hipEventDisableTiming);
      if (e != hipSuccess) {
        c->chr_ev = nullptr;
        return hip_fail(c, e, "two-pass event");
      }
    }
    if (c->chr_pending) {
      hipError_t e = hipStreamWaitEvent(s, c->chr_ev, 0);
      if (e != hipSuccess) return hip_fail(c, e, "two-pass ordering");
    }
  }
  const bool dyn_peak = c->params.peak_detect &&
                        (k.tonemap == H2S_TM_BT2390 || k.tonemap == H2S_TM_SPLINE || k.pipe == h2s::PIPE_LIBPLACEBO);
  // host frames: the chunk pipeline, with the dynamic peak too (its
  // statistics, IIR and curve records run on the device, stream-ordered per
  // chunk on the compute stream, so the state still advances frame by frame)
  if ((host_in || host_out) && nframes > 1 && !c->serial_host)
    return process_pipelined(c, k, in, out, din, dout, nframes, fast, vec, out8, s, dyn_peak);
  if (host_in) {
    hipError_t e = copy_frames(&din, in, nframes, s);
    if (e != hipSuccess) return queued_exit(c, s, hip_fail(c, e, "host->device copy"));
  }
  const int slot = (int)(c->ev_count % kEvRing);
  if (c->timing) {
    if (!c->ev0[slot]) {
      hipEventCreate(&c->ev0[slot]);
      hipEventCreate(&c->ev1[slot]);
    }
    hipEventRecord(c->ev0[slot], s);
  }
  hipError_t e;
  if (dyn_peak) {
    if ((rc = run_dynamic_peak(c, k, fast, vec, out8, nframes, s))) return queued_exit(c, s, rc);
    e = hipSuccess;
  } else {
    e = launch_chain(c, k, fast, vec, out8, nframes, s);
  }
  if (e == hipSuccess && c->fail_after_launch) {
    c->fail_after_launch = false;
    return queued_exit(c, s, fail(c, H2S_E_HIP, "injected failure after the launch (H2S_OPT_TEST_FAIL_AFTER_LAUNCH)"));
  }
  if (e != hipSuccess) return queued_exit(c, s, hip_fail(c, e, "kernel launch"));
  if (c->timing) {
    hipEventRecord(c->ev1[slot], s);
    c->ev_count++;
  }
  if (host_out) {
    e = copy_frames(out, &dout, nframes, s);
    if (e != hipSuccess) return queued_exit(c, s, hip_fail(c, e, "device->host copy"));
  }
  if (two_pass) {
    if ((e = hipEventRecord(c->chr_ev, s)) != hipSuccess) return queued_exit(c, s, hip_fail(c, e, "two-pass event"));
    c->chr_pending = true;
  }
  if (host_in || host_out) {
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return queued_exit(c, s, hip_fail(c, e, "stream synchronize"));
    return 0;
  }
  return note_launch(c, s);
}

int h2s_debug_float(h2s_ctx* c, const h2s_frames* in, int stage, float* out_rgb, int out_location,
                    void* hip_stream) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  if (stage < H2S_STAGE_LINEAR || stage > H2S_STAGE_YUV) return fail(c, H2S_E_INVALID_ARG, "bad stage");
  if (!out_rgb) return fail(c, H2S_E_INVALID_ARG, "out_rgb is NULL");
  KParams k;
  int rc = prepare(c, &k);
  if (rc) return rc;
  if ((rc = check_frames(c, in, c->params.bits_in, "input"))) return rc;
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)hip_stream;
  const size_t npx = (size_t)in->width * in->height, ob = npx * 3 * sizeof(float);
  // scratch: a tight device copy of the input (host input), the float planes
  // (host output) and one output frame for the tile kernel's own stores
  h2s_frames fo{};
  fo.width = in->width, fo.height = in->height, fo.bits = c->params.bits_out, fo.location = H2S_LOC_DEVICE;
  const size_t ib = in->location == H2S_LOC_HOST ? (frame_bytes(in) + 255) / 256 * 256 : 0;
  const size_t fb = (frame_bytes(&fo) + 255) / 256 * 256, pb = out_location == H2S_LOC_HOST ? ob : 0;
  void* scratch = nullptr;
  hipError_t e = hipMalloc(&scratch, ib + fb + pb + 256);
  if (e != hipSuccess) return fail(c, H2S_E_OOM, "debug alloc");
  uint8_t* base = (uint8_t*)scratch;
  h2s_frames din = *in;
  if (in->location == H2S_LOC_HOST) {
    din = tight(in, base);
    if ((e = copy_frames(&din, in, 1, s)) != hipSuccess) {
      hipFree(scratch);
      return hip_fail(c, e, "debug copy");
    }
  }
  fo = tight(&fo, base + ib);
  float* dout = out_location == H2S_LOC_HOST ? (float*)(base + ib + fb) : out_rgb;
  fill_geometry(&k, &din, &fo, 1);
  const bool out8 = c->params.bits_out == 8;
  const int path = choose_path(c, k, &din, &fo, out8);
  // the generic debug kernel covers every pixel; on the tile path the tile
  // kernel's debug instance then rewrites the tile columns with its own values
  e = h2s::launch_debug(k, stage, dout, s);
  if (e == hipSuccess && (path == H2S_PATH_TILE || path == H2S_PATH_TILE_TAIL)) {
    if (k.lut_enabled && (rc = ensure_lut_yuv(c, k, s))) {
      hipStreamSynchronize(s);
      hipFree(scratch);
      return rc;
    }
    e = launch_chain(c, k, true, false, out8, 1, s, nullptr, false, stage, dout);
  }
  if (e == hipSuccess && out_location == H2S_LOC_HOST) e = hipMemcpyAsync(out_rgb, dout, ob, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  hipStreamSynchronize(s);
  hipFree(scratch);
  if (e != hipSuccess) return hip_fail(c, e, "debug kernel");
  return 0;
}

int h2s_set_option(h2s_ctx* c, int key, int64_t value) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  switch (key) {
    case H2S_OPT_FAST_PATH:
      c->fast_enabled = value != 0;
      return 0;
    case H2S_OPT_TILES_PER_BLOCK:
      if (value < 1 || value > 64) return fail(c, H2S_E_INVALID_ARG, "tiles per block must be in [1, 64]");
      c->tiles_per_block = (int)value;
      return 0;
    case H2S_OPT_HOST_SERIAL:
      c->serial_host = value != 0;
      return 0;
    case H2S_OPT_LP_EXACT:
      c->lp_exact = value != 0;
      return 0;
    case 4:   // reserved: H2S_OPT_LP_EXACT's key in ABI 3.3
      return fail(c, H2S_E_INVALID_ARG, "option 4 is reserved (H2S_OPT_LP_EXACT is option 5 since ABI 3.4)");
    case H2S_OPT_TEST_FAIL_AFTER_LAUNCH:
      c->fail_after_launch = value != 0;
      return 0;
    case H2S_OPT_TEST_PEAK_FORM:
      c->peak_form = (int)value;
      return 0;
    case H2S_OPT_TEST_PEAK_BLOCKS:
      if (value < 1 || value > h2s::PEAK_BLOCKS_MAX) return fail(c, H2S_E_INVALID_ARG, "peak blocks must be in [1, 256]");
      c->peak_blocks = (int)value;
      return 0;
    case H2S_OPT_TEST_PEAK_CHUNK:
      if (value < 0 || value > 4096) return fail(c, H2S_E_INVALID_ARG, "peak chunk must be in [0, 4096]");
      c->peak_chunk = (int)value;
      return 0;
    default:
      return fail(c, H2S_E_INVALID_ARG, "unknown option");
  }
}

int h2s_query_path(h2s_ctx* c, const h2s_frames* in, const h2s_frames* out) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  KParams k;
  int rc = prepare(c, &k);
  if (rc) return rc;
  if ((rc = check_frames(c, in, c->params.bits_in, "input"))) return rc;
  if ((rc = check_frames(c, out, c->params.bits_out, "output"))) return rc;
  // host sets are staged into tight device copies, whose alignment decides
  h2s_frames din = *in, dout = *out;
  uint8_t* fake = (uint8_t*)(uintptr_t)4096;
  if (in->location == H2S_LOC_HOST) din = tight(in, fake);
  if (out->location == H2S_LOC_HOST) dout = tight(out, fake);
  return choose_path(c, k, &din, &dout, c->params.bits_out == 8);
}

// ---- preview ---------------------------------------------------------------

int h2s_preview_size(int in_w, int in_h, int box_w, int box_h, int* out_w, int* out_h) {
  if (in_w <= 0 || in_h <= 0 || box_w <= 0 || box_h <= 0 || !out_w || !out_h)
    return fail(nullptr, H2S_E_INVALID_ARG, "preview sizes must be positive");
  // libavfilter scale_eval: av_rescale (round half away from zero) of the
  // box by the input aspect, then min with the box (decrease)
  auto rescale = [](long long a, long long b, long long c) { return (a * b + c / 2) / c; };
  const long long tw = rescale(box_h, in_w, in_h), th = rescale(box_w, in_h, in_w);
  *out_w = (int)(tw < box_w ? tw : box_w);
  *out_h = (int)(th < box_h ? th : box_h);
  if (*out_w < 1) *out_w = 1;
  if (*out_h < 1) *out_h = 1;
  return 0;
}

namespace {
// swscale SWS_BICUBIC with its default parameters B = 0, C = 0.6
double bicubic(double x) {
  const double B = 0.0, C = 0.6;
  x = fabs(x);
  if (x < 1.0) return ((12 - 9 * B - 6 * C) * x * x * x + (-18 + 12 * B + 6 * C) * x * x + (6 - 2 * B)) / 6.0;
  if (x < 2.0) return ((-B - 6 * C) * x * x * x + (6 * B + 30 * C) * x * x + (-12 * B - 48 * C) * x + (8 * B + 24 * C)) / 6.0;
  return 0.0;
}

// per output index: first source tap and T normalised weights (centre-aligned
// sampling; the kernel widens by the ratio when downscaling)
int resize_taps(int src, int dst, std::vector<float>* w, std::vector<int>* start) {
  const double scale = (double)src / dst, fw = scale > 1.0 ? scale : 1.0;
  const int T = (int)ceil(4.0 * fw) + 1;
  w->assign((size_t)dst * T, 0.0f);
  start->assign(dst, 0);
  for (int o = 0; o < dst; o++) {
    const double c = (o + 0.5) * scale - 0.5;
    const int s0 = (int)floor(c - 2.0 * fw) + 1;
    double sum = 0.0, tmp[64];
    for (int i = 0; i < T && i < 64; i++) sum += (tmp[i] = bicubic((s0 + i - c) / fw));
    for (int i = 0; i < T && i < 64; i++) (*w)[(size_t)o * T + i] = (float)(tmp[i] / sum);
    (*start)[o] = s0;
  }
  return T;
}
}  // namespace

int h2s_preview_rgb24_batch(h2s_ctx* c, const h2s_frames* in, int nframes, uint8_t* rgb, int64_t rgb_linesize,
                            int64_t rgb_frame_pitch, int out_w, int out_h, double display_gamma, int rgb_location,
                            void* hip_stream) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  if (nframes < 1) return fail(c, H2S_E_INVALID_ARG, "nframes must be >= 1");
  if (!rgb || out_w <= 0 || out_h <= 0 || rgb_linesize < 3LL * out_w ||
      (nframes > 1 && rgb_frame_pitch < rgb_linesize * out_h))
    return fail(c, H2S_E_INVALID_ARG, "bad RGB output geometry");
  if (!(display_gamma > 0.0)) return fail(c, H2S_E_INVALID_ARG, "display gamma must be > 0");
  if (!c->params_set) return fail(c, H2S_E_INVALID_ARG, "h2s_set_params was not called");
  if (c->params.bits_out != 8)
    return fail(c, H2S_E_INVALID_ARG, "preview needs params.bits_out == 8 (the chain's yuv420p)");
  int rc = check_frames(c, in, c->params.bits_in, "input");
  if (rc) return rc;
  const int W = in->width, H = in->height;
  const bool scale = out_w != W || out_h != H;
  if (scale && (out_w > 4 * 8192 || out_h > 4 * 8192 || (double)W / out_w > 12.0 || (double)H / out_h > 12.0))
    return fail(c, H2S_E_UNSUPPORTED, "preview resize ratio out of range");
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)hip_stream;
  // scratch: chain output (yuv420p), resized planes, tap tables, RGB, gamma LUT
  const int ow2 = (out_w + 1) / 2, oh2 = (out_h + 1) / 2;
  std::vector<float> wx, wy, wcx, wcy;
  std::vector<int> sx, sy, scx, scy;
  int T = 0, Tc = 0;
  if (scale) {
    T = resize_taps(W, out_w, &wx, &sx);
    const int Ty = resize_taps(H, out_h, &wy, &sy);
    Tc = resize_taps(W / 2, ow2, &wcx, &scx);
    const int Tcy = resize_taps(H / 2, oh2, &wcy, &scy);
    if (Ty != T || Tcy != Tc) {  // one T per plane: recompute on the wider support
      const int Tm = T > Ty ? T : Ty, Tcm = Tc > Tcy ? Tc : Tcy;
      auto widen = [](std::vector<float>* w, int n, int t, int tn) {
        std::vector<float> o((size_t)n * tn, 0.0f);
        for (int i = 0; i < n; i++)
          for (int k = 0; k < t; k++) o[(size_t)i * tn + k] = (*w)[(size_t)i * t + k];
        *w = o;
      };
      if (T < Tm) widen(&wx, out_w, T, Tm);
      if (Ty < Tm) widen(&wy, out_h, Ty, Tm);
      if (Tc < Tcm) widen(&wcx, ow2, Tc, Tcm);
      if (Tcy < Tcm) widen(&wcy, oh2, Tcy, Tcm);
      T = Tm, Tc = Tcm;
    }
  }
  uint8_t glut[256];
  for (int i = 0; i < 256; i++) {
    // PIL point() with round() of pow(i/255, 1/gamma)*255 (round half to even)
    const double v = display_gamma == 1.0 ? (double)i : pow(i / 255.0, 1.0 / display_gamma) * 255.0;
    const double r = nearbyint(v);
    glut[i] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
  }
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t n = (size_t)nframes;
  const size_t yfp = (size_t)W * H * 3 / 2;                             // tight yuv420p frame
  const size_t sfp = (size_t)out_w * out_h + 2 * (size_t)ow2 * oh2;    // one resized frame
  const size_t yuv_b = al(yfp * n), syuv_b = scale ? al(sfp * n) : 0;
  const size_t tab_b = scale ? al((wx.size() + wy.size() + wcx.size() + wcy.size()) * 4) +
                                   al((sx.size() + sy.size() + scx.size() + scy.size()) * 4)
                             : 0;
  const size_t rgb_b = rgb_location == H2S_LOC_HOST ? al((size_t)out_w * 3 * out_h * n) : 0;
  const size_t need = yuv_b + syuv_b + tab_b + rgb_b + 256;
  if (need > c->prev_bytes) {
    if (c->d_prev) {
      // a previous preview's kernels may still read the old scratch
      drain_launches(c);
      hipStreamSynchronize(s);
      hipFree(c->d_prev);
    }
    c->d_prev = nullptr;
    c->prev_bytes = 0;
    if (hipMalloc(&c->d_prev, need) != hipSuccess) {
      c->d_prev = nullptr;
      return fail(c, H2S_E_OOM, "preview scratch allocation failed");
    }
    c->prev_bytes = need;
  }
  uint8_t* base = (uint8_t*)c->d_prev;
  h2s_frames y8{};
  y8.width = W, y8.height = H, y8.bits = 8, y8.location = H2S_LOC_DEVICE;
  y8 = tight(&y8, base);
  if (c->params.peak_detect) {
    // libplacebo branch: the reference converts each preview frame in its own
    // ffmpeg run (extract_frames_with_gpu_conversion_batch loops
    // extract_frame_with_gpu_conversion, src/utils.py:803-824), so peak
    // detection starts afresh on every frame: one launch per frame, state
    // reset in between.  The context's own state (a conversion sequence the
    // caller may be in the middle of) is saved first and restored afterwards,
    // all stream-ordered on s
    if ((rc = ensure_peak_state(c)) || (rc = peak_order(c, s))) return rc;
    const size_t pb = sizeof(h2s::PeakState);
    hipError_t e = hipMemcpyAsync(c->d_pk + 1, c->d_pk, pb, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return hip_fail(c, e, "peak state save");
    // every exit after the save queues the restore first (best effort)
    auto restored = [&](int code) {
      (void)hipMemcpyAsync(c->d_pk, c->d_pk + 1, pb, hipMemcpyDeviceToDevice, s);
      (void)peak_done(c, s);
      return code;
    };
    for (int f = 0; f < nframes; f++) {
      h2s_frames fi = *in, fo = y8;
      for (int k = 0; k < 3; k++) {
        fi.data[k] = (uint8_t*)in->data[k] + (long long)f * in->frame_pitch[k];
        fo.data[k] = (uint8_t*)y8.data[k] + (long long)f * y8.frame_pitch[k];
      }
      if ((e = hipMemsetAsync(c->d_pk, 0, pb, s)) != hipSuccess)
        return restored(queued_exit(c, s, hip_fail(c, e, "peak state reset")));
      if ((rc = h2s_process(c, &fi, &fo, 1, hip_stream))) return restored(rc);
    }
    if ((e = hipMemcpyAsync(c->d_pk, c->d_pk + 1, pb, hipMemcpyDeviceToDevice, s)) != hipSuccess)
      return queued_exit(c, s, hip_fail(c, e, "peak state restore"));
    if ((rc = peak_done(c, s))) return queued_exit(c, s, rc);
  } else if ((rc = h2s_process(c, in, &y8, nframes, hip_stream))) {  // one launch for the batch
    return rc;
  }
  hipError_t e = hipSuccess;
  const uint8_t *yp = (const uint8_t*)y8.data[0], *up = (const uint8_t*)y8.data[1], *vp = (const uint8_t*)y8.data[2];
  long long yls = W, cls = W / 2, fp = (long long)yfp;
  uint8_t* p = base + yuv_b;
  if (scale) {
    uint8_t* sy_ = p;
    uint8_t* su_ = p + (size_t)out_w * out_h;
    uint8_t* sv_ = su_ + (size_t)ow2 * oh2;
    uint8_t* t = p + syuv_b;
    float* dwx = (float*)t;
    float* dwy = dwx + wx.size();
    float* dwcx = dwy + wy.size();
    float* dwcy = dwcx + wcx.size();
    int* dsx = (int*)(t + al((wx.size() + wy.size() + wcx.size() + wcy.size()) * 4));
    int* dsy = dsx + sx.size();
    int* dscx = dsy + sy.size();
    int* dscy = dscx + scx.size();
    struct {
      void* d;
      const void* h;
      size_t b;
    } up_[8] = {{dwx, wx.data(), wx.size() * 4},   {dwy, wy.data(), wy.size() * 4},   {dwcx, wcx.data(), wcx.size() * 4},
                {dwcy, wcy.data(), wcy.size() * 4}, {dsx, sx.data(), sx.size() * 4},   {dsy, sy.data(), sy.size() * 4},
                {dscx, scx.data(), scx.size() * 4}, {dscy, scy.data(), scy.size() * 4}};
    for (auto& u : up_)
      if (e == hipSuccess) e = hipMemcpyAsync(u.d, u.h, u.b, hipMemcpyHostToDevice, s);
    const long long sp = (long long)sfp;
    if (e == hipSuccess)
      e = h2s::launch_resize_u8(yp, W, H, W, fp, sy_, out_w, out_h, out_w, sp, dwx, dsx, dwy, dsy, T, nframes, s);
    if (e == hipSuccess)
      e = h2s::launch_resize_u8(up, W / 2, H / 2, W / 2, fp, su_, ow2, oh2, ow2, sp, dwcx, dscx, dwcy, dscy, Tc,
                                nframes, s);
    if (e == hipSuccess)
      e = h2s::launch_resize_u8(vp, W / 2, H / 2, W / 2, fp, sv_, ow2, oh2, ow2, sp, dwcx, dscx, dwcy, dscy, Tc,
                                nframes, s);
    yp = sy_, up = su_, vp = sv_, yls = out_w, cls = ow2, fp = sp;
  }
  uint8_t* dglut = base + need - 256;
  const bool host = rgb_location == H2S_LOC_HOST;
  uint8_t* drgb = host ? base + yuv_b + syuv_b + tab_b : rgb;
  const long long drls = host ? 3LL * out_w : rgb_linesize;
  const long long drfp = host ? 3LL * out_w * out_h : rgb_frame_pitch;
  if (e == hipSuccess) e = hipMemcpyAsync(dglut, glut, 256, hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = h2s::launch_yuv8_rgb24(yp, yls, up, vp, cls, fp, out_w, out_h, drgb, drls, drfp, dglut, nframes, s);
  for (int f = 0; host && f < nframes && e == hipSuccess; f++)
    e = hipMemcpy2DAsync(rgb + (long long)f * rgb_frame_pitch, rgb_linesize, drgb + f * drfp, drls, 3 * (size_t)out_w,
                         out_h, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(c, e, "preview");
  return 0;
}

int h2s_preview_rgb24(h2s_ctx* c, const h2s_frames* in, uint8_t* rgb, int64_t rgb_linesize, int out_w, int out_h,
                      double display_gamma, int rgb_location, void* hip_stream) {
  return h2s_preview_rgb24_batch(c, in, 1, rgb, rgb_linesize, rgb_linesize * (int64_t)out_h, out_w, out_h,
                                 display_gamma, rgb_location, hip_stream);
}

int h2s_set_timing(h2s_ctx* c, int enabled) {
  if (!c) return fail(nullptr, H2S_E_INVALID_ARG, "ctx is NULL");
  c->timing = enabled != 0;
  c->ev_count = 0;
  return 0;
}

double h2s_kernel_ms(h2s_ctx* c, int count) {
  if (!c) return -1.0;
  if (count <= 0) {
    c->ev_count = 0;
    return 0.0;
  }
  DeviceGuard g(c->device);
  const long long avail = c->ev_count < kEvRing ? c->ev_count : kEvRing;
  if (count > avail) count = (int)avail;
  if (count == 0) return 0.0;
  double sum = 0.0;
  for (int i = 0; i < count; i++) {
    const int slot = (int)((c->ev_count - 1 - i) % kEvRing);
    if (hipEventSynchronize(c->ev1[slot]) != hipSuccess) return -1.0;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, c->ev0[slot], c->ev1[slot]) != hipSuccess) return -1.0;
    sum += ms;
  }
  return sum / count;
}

}  // extern "C"
