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
 * synchronises.
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

#define H2S_ABI_VERSION 1

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

/* Luma weights tonemap's desaturation uses (vf_tonemap reads the frame's
 * colorspace; after zscale's float RGB output that is AVCOL_SPC_RGB, whose
 * libavutil entry is {1,1,1}).  Switchable because it cannot be pinned
 * without the bundled ffmpeg. */
enum h2s_desat_luma {
  H2S_DESAT_LUMA_RGB = 0,    /* {1, 1, 1}                 */
  H2S_DESAT_LUMA_BT2020 = 1, /* {0.2627, 0.6780, 0.0593}  */
  H2S_DESAT_LUMA_BT709 = 2   /* {0.2126, 0.7152, 0.0722}  */
};

/* Where a frame set lives. */
enum h2s_location { H2S_LOC_DEVICE = 0, H2S_LOC_HOST = 1 };

/* Debug stages for h2s_debug_float (float RGB after each chain stage). */
enum h2s_stage {
  H2S_STAGE_LINEAR = 1,   /* after S1 zscale=t=linear:npl=100          */
  H2S_STAGE_TONEMAP = 2,  /* after S2 tonemap=                          */
  H2S_STAGE_GAMMA = 3,    /* after S3 zscale=t=bt709 (BT.1886 inverse)  */
  H2S_STAGE_LUT = 4       /* after S4 lut3d=interp=tetrahedral          */
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
  int32_t reserved[4];
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
 * Device->device runs asynchronously; any host-resident set is staged
 * through context-owned device buffers and the call returns after the copy
 * back (PCIe-inclusive path). */
int h2s_process(h2s_ctx *ctx, const h2s_frames *in, const h2s_frames *out,
                int nframes, void *hip_stream);

/* Debug/parity: float RGB (planar, 3*w*h floats: R plane, G plane, B plane)
 * of frame 0 after `stage` (enum h2s_stage), written to out_rgb (host or
 * device per out_location).  Synchronous. */
int h2s_debug_float(h2s_ctx *ctx, const h2s_frames *in, int stage,
                    float *out_rgb, int out_location, void *hip_stream);

/* ---- dynamic peak (params.peak_detect, BT.2390 / spline) -----------------
 * h2s_peak_reset: forget the smoothing state (a new sequence / scene cut).
 * h2s_peak_state: the smoothed PQ-domain max / average after the last
 *   processed frame, the source peak (units of npl) it gave, and the number
 *   of frames folded in since the reset.  Any pointer may be NULL. */
int h2s_peak_reset(h2s_ctx *ctx);
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
 *   rgb_location.  Synchronous. */
int h2s_preview_size(int in_w, int in_h, int box_w, int box_h, int *out_w, int *out_h);
int h2s_preview_rgb24(h2s_ctx *ctx, const h2s_frames *in, uint8_t *rgb, int64_t rgb_linesize,
                      int out_w, int out_h, double display_gamma, int rgb_location,
                      void *hip_stream);

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
