/*
 * h2s.h — C-ABI of libh2s, the MI355X-native HDR10/HLG -> SDR tone-mapping
 * hot path.  This is the drop-in boundary for the reference's CPU ffmpeg
 * filter chain.
 *
 * The reference (TORlN/HDR-to-SDR) has no native FFI of its own: its hot path
 * is the filtergraph string
 *
 *   zscale=t=linear:npl=100,tonemap={tm},zscale=t=bt709:m=bt709:r=tv,
 *   lut3d=file={lut}:interp=tetrahedral,setparams=...bt709,eq=gamma={g}
 *
 * (src/utils.py:38-42), formatted by ffmpeg_command._filter_args
 * (src/ffmpeg_command.py:227-247) and executed frame by frame inside an ffmpeg
 * child process (src/conversion.py:209-224).  Each entry point below names
 * the reference interface it replaces.  All signatures use plain C types:
 * pointers, sizes and POD structs — no torch or HIP types leak through.
 *
 * Threading: every function is callable from any thread.  A context must not
 * be used by two threads at once (one context per worker / GPU), and contexts
 * share no mutable global state.  h2s_process is asynchronous on the stream
 * it is given when both frame sets live in device memory; the caller
 * synchronises.  h2s_set_params and h2s_set_lut first wait for every launch
 * the context has queued (on any stream) to finish, so replacing the tables a
 * kernel in flight reads is safe; they wait on events recorded after the
 * context's own launches only, never on other contexts or on unrelated work
 * on the device.
 *
 * Errors: 0 on success, a negative H2S_E_* code otherwise; the message is
 * available from h2s_last_error(ctx) (or h2s_last_error(NULL) for failures
 * that happen before a context exists).  The Python host maps the codes to the
 * reference's exception types (ValueError / FileNotFoundError / RuntimeError,
 * src/ffmpeg_command.py:240-245, src/utils.py:185-186, src/utils.py:297-308).
 */
#ifndef H2S_H
#define H2S_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define H2S_ABI_VERSION 3
/* Minor revision within ABI 3 (h2s_abi_minor), for bindings that need to
 * detect additions and behaviour changes that keep every v3 signature:
 *   1: h2s_preview_rgb24_batch; the lp_p010 default TRUNCATE (the reference's
 *      format=p010 upload; 12-bit libplacebo-branch output changes);
 *   2: h2s_process with params.peak_detect is asynchronous on its stream (the
 *      peak statistics, smoothing and curve constants run on the device);
 *      h2s_peak_state / _reset / _feed wait for the context's queued work; a
 *      preview restores the context's peak state; the failure-injection test
 *      hook moved to the private option range (H2S_PRIVATE_TEST_HOOKS);
 *   3: H2S_OPT_LP_EXACT (then key 4);
 *   4: H2S_OPT_LP_EXACT moves to key 5 and key 4 is reserved (H2S_E_INVALID_ARG:
 *      a 3.0 / 3.1 client that set key 4 as the old failure-injection hook
 *      fails loudly instead of switching kernels); the libplacebo branch's
 *      exact path computes stages 1-3 in double precision (see below). */
#define H2S_ABI_MINOR 4

/* ---- error codes ------------------------------------------------------- */
#define H2S_OK 0
#define H2S_E_INVALID_ARG (-1)  /* bad pointer / size / enum value        */
#define H2S_E_UNSUPPORTED (-2)  /* valid request this build cannot serve  */
#define H2S_E_HIP (-3)          /* HIP runtime error (message has detail) */
#define H2S_E_OOM (-4)          /* device or host allocation failed       */
#define H2S_E_LUT_MISSING (-5)  /* lut_enabled but no LUT loaded          */
#define H2S_E_PARSE (-6)        /* malformed .cube / filter text          */

/* ---- enums ------------------------------------------------------------- */
/* Input transfer of the source frames (frame tag read by zscale t=linear). */
enum h2s_transfer { H2S_TRC_PQ = 0, H2S_TRC_HLG = 1 };

/* Tone-map operators.  NONE..MOBIUS are ffmpeg vf_tonemap's `tonemap=`
 * values (the reference exposes reinhard/mobius/hable, src/utils.py:16);
 * BT2390 and SPLINE are the GPU-only operators the reference reaches through
 * libplacebo's `tonemapping=` (GPU_ONLY_TONEMAPPERS, src/utils.py:62-73,
 * :392-471).  SPLINE's tm_param is libplacebo's spline contrast (NaN = 0.5,
 * range 0..1.5). */
enum h2s_tonemap {
  H2S_TM_NONE = 0,
  H2S_TM_LINEAR = 1,
  H2S_TM_GAMMA = 2,
  H2S_TM_CLIP = 3,
  H2S_TM_REINHARD = 4,
  H2S_TM_HABLE = 5,
  H2S_TM_MOBIUS = 6,
  H2S_TM_BT2390 = 7,
  H2S_TM_SPLINE = 8
};

/* Output quantisation.  COMPAT8 reproduces the reference CPU chain's 8-bit
 * bottleneck (eq is 8-bit only, so ffmpeg converts to yuv420p before it and
 * shifts up to the -pix_fmt afterwards, src/ffmpeg_command.py:355-360, :501).
 * NATIVE quantises directly to bits_out. */
enum h2s_mode { H2S_MODE_COMPAT8 = 0, H2S_MODE_NATIVE = 1 };

/* Luma weights tonemap's desaturation uses: vf_tonemap reads the frame's
 * colorspace tag -- bt2020nc if the first zscale (no m=) carries it through,
 * or, if colorspace negotiation retags the float RGB frame, the libavutil RGB
 * entry {1,1,1} (the default).  Switchable because it cannot be pinned
 * without the bundled ffmpeg: the reference's only
 * pixel pair was made on its libplacebo branch, where no vf_tonemap runs. */
enum h2s_desat_luma {
  H2S_DESAT_LUMA_RGB = 0,    /* {1, 1, 1}                 */
  H2S_DESAT_LUMA_BT2020 = 1, /* {0.2627, 0.6780, 0.0593}  */
  H2S_DESAT_LUMA_BT709 = 2   /* {0.2126, 0.7152, 0.0722}  */
};

/* Where a frame set lives. */
enum h2s_location { H2S_LOC_DEVICE = 0, H2S_LOC_HOST = 1 };

/* Debug stages for h2s_debug_float: three float planes per pixel.
 * 1..4: R, G, B after the stage.  5: the quantiser's inputs, before rounding:
 * plane 0 = luma code (16 + 219 Y) * 2^(q-8), planes 1/2 = the pixel's Cb / Cr
 * in code units, 224 * 2^(q-8) * C (the 4:2:0 sample is 128 * 2^(q-8) plus
 * the chroma filter over these), q = the quantisation depth. */
enum h2s_stage {
  H2S_STAGE_LINEAR = 1,   /* after S1 zscale=t=linear:npl=100          */
  H2S_STAGE_TONEMAP = 2,  /* after S2 tonemap=                          */
  H2S_STAGE_GAMMA = 3,    /* after S3 zscale=t=bt709 (BT.1886 inverse)  */
  H2S_STAGE_LUT = 4,      /* after S4 lut3d=interp=tetrahedral          */
  H2S_STAGE_YUV = 5       /* S6 quantiser inputs (see above)            */
};

/* S6 chroma 4:4:4 -> 4:2:0 filter of the implicit swscale conversion
 * (cannot be pinned without the bundled ffmpeg).
 * BOX: the 2x2 mean of the quad (centre siting).  BICUBIC: swscale's default
 * bicubic (B = 0, C = 0.6) decimation, chroma sited left horizontally (on the
 * even luma column) and centred vertically, edge-clamped. */
enum h2s_chroma_filter { H2S_CHROMA_BOX = 0, H2S_CHROMA_BICUBIC = 1 };

/* Rounding of the 8-bit quantiser (S6 yuv420p, or the libplacebo branch's
 * rgba download).  NONE: round half up.  ORDERED: swscale's 8x8 ordered
 * dither offsets (ff_dither_8x8_128 / 128 of an LSB) instead of +0.5. */
enum h2s_dither { H2S_DITHER_NONE = 0, H2S_DITHER_ORDERED = 1 };

/* S1 chroma upsampler edge rule: the sample the
 * bilinear 2-tap reads past the plane's edge (row -1 above the first chroma
 * row, row ch below the last, column cw right of the last; left-sited chroma
 * never reads column -1).  ZIMG: -1 mirrors to 1, ch / cw fold to the last
 * sample (the round-1 model).  REPLICATE: every edge repeats its last
 * sample.  MIRROR: every edge mirrors about its last sample (ch -> ch-2). */
enum h2s_chroma_edge { H2S_EDGE_ZIMG = 0, H2S_EDGE_REPLICATE = 1, H2S_EDGE_MIRROR = 2 };

/* Format between S3 and S4 on the CPU chain: which
 * pixel format ffmpeg negotiates between zscale=t=bt709 and lut3d.  FLOAT:
 * gbrpf32, lut3d's float path (the round-1 model).  RGB48: 16-bit R'G'B' --
 * zscale rounds to 16 bits, lut3d's 16-bit path reads q (1/65535) (N-1) and
 * truncates its output to 16 bits, swscale converts from there. */
enum h2s_lut_input { H2S_LUT_IN_FLOAT = 0, H2S_LUT_IN_RGB48 = 1 };

/* How the libplacebo branch applies its PQ-domain curve (BT.2390 / SPLINE)
 * to colour.  libplacebo is absent: PARITY UNPINNED.  IPT (default): the
 * curve maps the intensity I of IPT-PQ -- linear BT.2020 -> XYZ -> LMS
 * (Hunt-Pointer-Estevez, D65-normalised), PQ-encoded in absolute
 * luminance, I = 0.4 L' + 0.4 M' + 0.2 S' (Ebner-Fairchild) -- and keeps
 * P and T; libplacebo tone-maps in IPT since v6, and on the reference's own
 * before/after pair this fits best (tests/test_website_fixture.py).
 * MAX_RGB: gain curve(max RGB) / max RGB on R, G, B (the round-2 model). */
enum h2s_lp_tone { H2S_LP_TONE_IPT = 0, H2S_LP_TONE_MAX_RGB = 1 };

/* libplacebo branch: the open options of the reference's stage
 * `libplacebo=...:range=tv:peak_detect=1:format=rgba` (src/utils.py:445-449),
 * each a named model (SURVEY.md App. B style; PARITY UNPINNED, libplacebo and
 * vf_libplacebo are absent from the image).
 * h2s_lp_range: FULL = the rgba download carries full-range codes
 *   round(255 v) (libplacebo ignores range= for an RGB output); LIMITED =
 *   range=tv applies to the RGB output: round(16 + 219 v), which lut3d and
 *   the auto-scale to -pix_fmt then read as full-range RGB.
 * h2s_lp_dither: NONE = the 8-bit download rounds to nearest; ORDERED = a
 *   16 x 16 Bayer matrix offsets each code before the truncation (a stand-in
 *   for libplacebo's default dither, whose blue-noise texture is not
 *   restated: it measures how much the dither matters).
 * h2s_lp_p010: the upload prefix (src/utils.py:430-431).  TRUNCATE (the
 *   default since ABI v3.1: the reference's default `format=p010,hwupload`
 *   prefix) = the 10-bit p010 container drops a 12-bit input's two low bits
 *   (code & ~3); KEEP = the CUDA-interop `hwmap=derive_device=vulkan` prefix,
 *   which maps the decoder's frame without a format conversion, so 12-bit
 *   input reaches libplacebo at full precision.  10-bit input: no effect. */
enum h2s_lp_range { H2S_LP_RANGE_FULL = 0, H2S_LP_RANGE_LIMITED = 1 };
enum h2s_lp_dither { H2S_LP_DITHER_NONE = 0, H2S_LP_DITHER_ORDERED = 1 };
enum h2s_lp_p010 { H2S_LP_P010_KEEP = 0, H2S_LP_P010_TRUNCATE = 1 };

/* S8 8-bit -> bits_out expansion after eq. */
enum h2s_expand { H2S_EXPAND_SHIFT = 0, H2S_EXPAND_REPLICATE = 1 };

/* Which of the reference's two chains the parameters describe.
 * CPU_CHAIN: FFMPEG_CONVERT_FILTER (src/utils.py:38-42): zscale -> tonemap ->
 *   zscale -> lut3d (float) -> yuv420p -> eq -> -pix_fmt.
 * LIBPLACEBO: build_libplacebo_filter (src/utils.py:392-471) with the LUT on:
 *   libplacebo tone map (BT.2390, spline, or libplacebo's own reinhard /
 *   hable / mobius, which the reference also routes there with GPU tone
 *   mapping on) -> BT.1886 encode against the SDR
 *   target -> 8-bit rgba download -> lut3d's 8-bit path (truncating output) ->
 *   Y'CbCr at the output depth (gamma = 1; the chain has no eq) or, with
 *   eq=gamma, yuv420p -> eq -> -pix_fmt.  With the LUT off the branch keeps
 *   libplacebo's own BT.709 conversion and nv12 (8-bit) download.
 * AUTO: LIBPLACEBO for BT2390 / SPLINE (the reference's GPU-only operators
 *   exist only there), CPU_CHAIN otherwise. */
enum h2s_pipeline { H2S_PIPE_AUTO = 0, H2S_PIPE_CPU_CHAIN = 1, H2S_PIPE_LIBPLACEBO = 2 };

/* Context options (h2s_set_option). */
enum h2s_option {
  H2S_OPT_FAST_PATH = 1,       /* 1 (default): the tile kernel where it applies; 0: generic kernel only */
  H2S_OPT_TILES_PER_BLOCK = 2, /* tile kernel: 64x32 tiles one block walks (1..64, default 8)          */
  H2S_OPT_HOST_SERIAL = 3,     /* host frames: 1 = one H2D, kernel, D2H per call (no chunk pipeline)   */
  /* 4: reserved (H2S_E_INVALID_ARG; was H2S_OPT_LP_EXACT in ABI 3.3)                                  */
  H2S_OPT_LP_EXACT = 5         /* 1: the libplacebo branch on its exact path only (see below)           */
};
/* H2S_OPT_LP_EXACT: the libplacebo branch's 8-bit rgba download rounds a
 * float (255 x the BT.1886 encode).  The reference computes it in
 * libplacebo's float32 GLSL, so the restated reference is exact arithmetic;
 * the tile kernel (default, float32) lands within its stated error bound of
 * it and may round a code lying that close to a tie the other way (about
 * 0.1 % of codes; lut3d's 8-bit lattice step then spreads such a flip over a
 * few output steps).  With 1 the branch runs on the generic kernel's exact
 * path, stages 1-3 in double precision from the integer codes: output within
 * one step of the restated reference everywhere, at a multiple of the tile
 * kernel's time. */
/* Keys from H2S_OPT_PRIVATE_BASE up are the library's own test / debug hooks:
 * not part of the ABI, may change or vanish in any build. */
#define H2S_OPT_PRIVATE_BASE 0x7f000000
#ifdef H2S_PRIVATE_TEST_HOOKS
/* 1 = the next h2s_process call reports H2S_E_HIP right after queueing its
 * kernels (the error exits must still record the launch) */
#define H2S_OPT_TEST_FAIL_AFTER_LAUNCH (H2S_OPT_PRIVATE_BASE + 1)
/* peak statistics kernel form (A/B measurements): 0 = 32-pixel quad units (default), 1 = round 5's row chunks */
#define H2S_OPT_TEST_PEAK_FORM (H2S_OPT_PRIVATE_BASE + 2)
/* dynamic peak on the tile kernel: frames per pipelined chunk (0 = statistics for
 * the whole batch, then one conversion launch) */
#define H2S_OPT_TEST_PEAK_CHUNK (H2S_OPT_PRIVATE_BASE + 3)
/* peak statistics: blocks (partial records) per frame, 1..256 (default 64) */
#define H2S_OPT_TEST_PEAK_BLOCKS (H2S_OPT_PRIVATE_BASE + 4)
#endif

/* Kernel path h2s_process takes for a given frame pair (h2s_query_path). */
enum h2s_path {
  H2S_PATH_TILE = 1,       /* k_tile only (width % 64 == 0)                      */
  H2S_PATH_TILE_TAIL = 2,  /* k_tile + k_process on the width % 64 columns       */
  H2S_PATH_GENERIC = 3,    /* k_process                                          */
  H2S_PATH_TWO_PASS = 4    /* k_process per-pixel chroma + bicubic decimation    */
};

/* ---- parameters ---------------------------------------------------------
 * Mirrors the values FFMPEG_CONVERT_FILTER.format(gamma, tonemapper,
 * lut_path) bakes into the chain string (src/ffmpeg_command.py:246-247) plus
 * the chain's hard-coded options (npl=100, desat default, interp) and the
 * output -pix_fmt (src/ffmpeg_command.py:355-360).                        */
typedef struct h2s_params {
  int32_t transfer_in;  /* enum h2s_transfer                               */
  int32_t bits_in;      /* 10 or 12 (yuv420p10le / yuv420p12le)            */
  int32_t bits_out;     /* 8, 10 or 12 (yuv420p / 10le / 12le)             */
  int32_t tonemap;      /* enum h2s_tonemap                                */
  double tm_param;      /* tonemap=param; NaN = vf_tonemap default         */
  double desat;         /* tonemap=desat; reference uses default 2.0       */
  double peak;          /* tonemap=peak; 0 = auto (side data / default)    */
  double npl;           /* zscale npl; reference: 100                      */
  double gamma;         /* eq=gamma; reference: ConversionRequest.gamma    */
  double maxcll;        /* frame side data MaxCLL (nits), 0 = absent       */
  double mastering_max; /* mastering display max luminance, 0 = absent     */
  int32_t lut_enabled;  /* 1: lut3d stage; 0: closed-form BT.2020->709     */
  int32_t mode;         /* enum h2s_mode                                   */
  int32_t desat_luma;   /* enum h2s_desat_luma                             */
  int32_t peak_detect;  /* BT.2390 / SPLINE: 1 = per-frame detected,
                         * temporally smoothed source peak (and, for SPLINE,
                         * average: the knee) (libplacebo peak_detect=1,
                         * src/utils.py:448); state lives in the context   */
  /* [EXT] switches the bundled ffmpeg would settle */
  int32_t chroma_filter; /* enum h2s_chroma_filter (S6)                     */
  int32_t dither;        /* enum h2s_dither (8-bit quantiser)               */
  int32_t expand;        /* enum h2s_expand (S8)                            */
  int32_t pipeline;      /* enum h2s_pipeline                               */
  /* libplacebo branch (BT.2390 / SPLINE); NaN = that branch's default      */
  double knee_offset;    /* BT.2390 knee offset: ks = (1+o) maxLum - o;
                          * libplacebo default 1.0, ITU-R BT.2390 0.5      */
  double target_black;   /* SDR target black (nits); NaN: LIBPLACEBO =
                          * white / 1000 (libplacebo's SDR contrast),
                          * CPU_CHAIN = 0 (no black-point adaptation)      */
  double target_white;   /* SDR target white (nits); NaN: LIBPLACEBO = 203
                          * (libplacebo's SDR white, BT.2408), CPU_CHAIN =
                          * npl                                            */
  int32_t chroma_edge;   /* enum h2s_chroma_edge (S1)                       */
  int32_t lut_input;     /* enum h2s_lut_input (S3 -> S4, CPU chain)        */
  int32_t lp_tone;       /* enum h2s_lp_tone (libplacebo branch)            */
  /* ABI v3: libplacebo branch options (enums above) */
  int32_t lp_range;      /* enum h2s_lp_range                               */
  int32_t lp_dither;     /* enum h2s_lp_dither                              */
  int32_t lp_p010;       /* enum h2s_lp_p010                                */
  int32_t reserved[2];   /* keeps the doubles below 8-byte aligned        */
  /* peak_detect=1 (libplacebo's pl_peak_detect_params as vf_libplacebo sets
   * them; NaN = vf_libplacebo's option defaults, in brackets):            */
  double pd_smoothing;   /* IIR smoothing period, frames [100]              */
  double pd_scene_low;   /* scene-change thresholds on the frame average,   */
  double pd_scene_high;  /*   % of the PQ range [5.5, 10]                   */
  double pd_percentile;  /* detected peak = this percentile of per-pixel
                          * PQ(max R,G,B); 100 = the maximum [99.995]       */
  double pd_min_peak;    /* lower bound on the detected peak, relative to
                          * the SDR target white [1.0]                      */
} h2s_params;

/* A batch of planar 4:2:0 frames (yuv420p / yuv420p10le / yuv420p12le).
 * Samples are uint8 when bits == 8, else little-endian uint16 holding the
 * value in the low bits (ffmpeg's *le layouts).  Frame f, plane p, row r
 * starts at data[p] + f*frame_pitch[p] + r*linesize[p] (bytes).          */
typedef struct h2s_frames {
  void *data[3];
  int64_t linesize[3];
  int64_t frame_pitch[3];
  int32_t width;    /* luma width  (even)  */
  int32_t height;   /* luma height (even)  */
  int32_t bits;     /* 8, 10 or 12         */
  int32_t location; /* enum h2s_location   */
} h2s_frames;

typedef struct h2s_ctx h2s_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
int h2s_abi_version(void);
int h2s_abi_minor(void);   /* H2S_ABI_MINOR of the loaded library */

/* Replaces spawning the ffmpeg child (src/conversion.py:209-224) and the
 * filter-graph setup it performs.  device = HIP device ordinal (the reference
 * always uses device 0: src/utils.py:99, src/ffmpeg_command.py:187). */
int h2s_create(int device, h2s_ctx **out);
void h2s_destroy(h2s_ctx *ctx);

/* Message for the last failure on ctx (or the calling thread when ctx is
 * NULL).  Never NULL; "" when there was none. */
const char *h2s_last_error(const h2s_ctx *ctx);

/* ---- LUT (lut3d=file=..., src/utils.py:40, :212-225) --------------------
 * rgb: n^3 float triples in .cube order (red fastest, then green, then blue),
 * i.e. exactly the order tools/generate_lut.py:97-109 writes.  The context
 * keeps its own device copy. */
int h2s_set_lut(h2s_ctx *ctx, const float *rgb, int n);

/* ---- params (FFMPEG_CONVERT_FILTER.format, src/utils.py:38-42) ----------- */
void h2s_params_default(h2s_params *p);
int h2s_set_params(h2s_ctx *ctx, const h2s_params *p);

/* ---- per-frame execution (the ffmpeg filter_frame loop) ------------------
 * Processes nframes frames from `in` into `out`.  Both sets must have the
 * same width/height; in->bits == params.bits_in, out->bits ==
 * params.bits_out.  hip_stream is a hipStream_t (NULL = default stream).
 * Device->device runs asynchronously, with params.peak_detect too (the peak
 * statistics, the smoothing and the per-frame curves are queued on the same
 * stream, ABI 3.2); any host-resident set is staged through context-owned
 * device buffers and the call returns after the copy back (PCIe-inclusive
 * path). */
int h2s_process(h2s_ctx *ctx, const h2s_frames *in, const h2s_frames *out,
                int nframes, void *hip_stream);

/* Debug/parity: three float planes (3*w*h floats) of frame 0 after `stage`
 * (enum h2s_stage), written to out_rgb (host or device per out_location).
 * Computed by the kernel h2s_process would use for this frame: the tile
 * kernel's own arithmetic (a debug instance of it) on the tile path, the
 * generic kernel otherwise (h2s_query_path; H2S_OPT_FAST_PATH = 0 forces the
 * generic one).  With peak_detect the curve uses the static peak (the
 * parameters' resolved peak), not the context's smoothed state: the debug
 * planes are a per-frame check of the arithmetic and leave that state
 * untouched.  Synchronous. */
int h2s_debug_float(h2s_ctx *ctx, const h2s_frames *in, int stage,
                    float *out_rgb, int out_location, void *hip_stream);

/* ---- options and introspection ------------------------------------------
 * h2s_set_option: enum h2s_option.  h2s_query_path: the enum h2s_path that
 * h2s_process(ctx, in, out, ...) would take with the current params, LUT and
 * options (negative H2S_E_* on invalid input). */
int h2s_set_option(h2s_ctx *ctx, int key, int64_t value);
int h2s_query_path(h2s_ctx *ctx, const h2s_frames *in, const h2s_frames *out);

/* ---- dynamic peak (params.peak_detect, BT.2390 / spline) -----------------
 * h2s_peak_reset: forget the smoothing state (a new sequence / scene cut).
 * h2s_peak_state: the smoothed PQ-domain max / average after the last
 *   processed frame, the source peak (units of npl) it gave, and the number
 *   of frames folded in since the reset.  Any pointer may be NULL.
 * The state lives on the device and is updated in stream order by the
 * h2s_process calls that use it; h2s_peak_reset / _feed / _state first wait
 * for this context's queued work, then act synchronously. */
int h2s_peak_reset(h2s_ctx *ctx);
/* Frame-sharded runs (hdr2sdr/dist.py): the smoothing is a recurrence over
 * the whole sequence, so a rank that owns frames [a, b) first needs the
 * state frames [0, a) leave.  h2s_peak_stats: the per-frame statistics
 * h2s_process would fold in (max and mean of PQ(max R,G,B)), for device
 * frames, without converting them.  h2s_peak_feed: fold n frames' statistics
 * into the state in order, as h2s_process does.  Gathering every rank's
 * statistics and feeding the preceding ones makes the sharded output equal
 * to the sequential one. */
int h2s_peak_stats(h2s_ctx *ctx, const h2s_frames *in, int nframes, double *fmax, double *favg, void *hip_stream);
int h2s_peak_feed(h2s_ctx *ctx, const double *fmax, const double *favg, int n);
int h2s_peak_state(const h2s_ctx *ctx, double *max_pq, double *avg_pq, double *peak, int64_t *frames);

/* ---- preview (src/utils.py:719-765 extract_frame_with_conversion, the
 * GUI's adjust_gamma src/preview.py:108-117) ------------------------------
 * h2s_preview_size: the size FFMPEG_FILTER's trailing
 *   scale=W:H:force_original_aspect_ratio=decrease (src/utils.py:46-49) gives
 *   an in_w x in_h frame in a box_w x box_h box (PREVIEW_SIZE = 3840x2160,
 *   src/preview.py:29); upscales too, as ffmpeg's scale does.
 * h2s_preview_rgb24: frame 0 of `in` through the chain (ctx params; bits_out
 *   must be 8: the yuv420p the PNG encoder reads), the bicubic (B=0, C=0.6)
 *   resize to out_w x out_h when that differs from the frame size, BT.709
 *   limited Y'CbCr -> full-range RGB24 (nearest chroma), then the display
 *   gamma LUT round(255 (i/255)^(1/gamma)) on R, G, B (1.0 = identity).
 *   rgb: out_h rows of out_w*3 bytes, rgb_linesize apart, host or device per
 *   rgb_location.  Synchronous.
 * h2s_preview_rgb24_batch: the same for nframes frames of `in` (one size)
 *   into nframes RGB images rgb_frame_pitch bytes apart — the reference's
 *   batched preview (extract_frames_with_conversion_batch /
 *   extract_frames_with_gpu_conversion_batch, src/utils.py:617-626,
 *   :668-716, :803-824).  The CPU chain runs the batch as one tone-map
 *   launch; with params.peak_detect (the libplacebo branch) each frame starts
 *   from a fresh peak state, as each of the reference's per-frame ffmpeg runs
 *   does, and the context's own peak state is restored afterwards.  The resize and RGB kernels take the whole batch in one launch each.
 *   h2s_preview_rgb24 == the batch call with nframes = 1. */
int h2s_preview_size(int in_w, int in_h, int box_w, int box_h, int *out_w, int *out_h);
int h2s_preview_rgb24(h2s_ctx *ctx, const h2s_frames *in, uint8_t *rgb, int64_t rgb_linesize,
                      int out_w, int out_h, double display_gamma, int rgb_location,
                      void *hip_stream);
int h2s_preview_rgb24_batch(h2s_ctx *ctx, const h2s_frames *in, int nframes, uint8_t *rgb,
                            int64_t rgb_linesize, int64_t rgb_frame_pitch, int out_w, int out_h,
                            double display_gamma, int rgb_location, void *hip_stream);

/* ---- .cube helpers (tools/generate_lut.py:28-119; lut3d's .cube parser) --
 * h2s_cube_generate: the BT.2020->BT.709 lattice, n^3 triples, .cube order,
 *   rounded exactly as the "%.6f" text the reference writes, then parsed to
 *   float32 (what lut3d holds after reading the file).
 * h2s_cube_format: the file text, byte-identical to
 *   '\n'.join(generate_cube_lines(n)) + '\n'.  Returns the byte count
 *   needed (excluding NUL); writes at most cap bytes.
 * h2s_cube_parse: parses .cube text (LUT_3D_SIZE header, comments, optional
 *   DOMAIN_MIN/MAX of 0/1) into float32 triples; *n_out gets the size.  Pass
 *   rgb=NULL to query the size first. */
int h2s_cube_generate(int n, float *rgb);
int64_t h2s_cube_format(int n, char *buf, int64_t cap);
int h2s_cube_parse(const char *text, int64_t len, float *rgb, int64_t cap_floats,
                   int *n_out);

/* Kernel-duration probe for bench.py: average device time (ms) of the last
 * `count` h2s_process launches recorded with HIP events on the launch stream
 * since the last reset (count <= 0 resets the record and returns 0). */
double h2s_kernel_ms(h2s_ctx *ctx, int count);
int h2s_set_timing(h2s_ctx *ctx, int enabled);

#ifdef __cplusplus
}
#endif
#endif /* H2S_H */
