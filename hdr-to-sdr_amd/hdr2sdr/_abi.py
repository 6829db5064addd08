"""ctypes binding of libh2s (include/h2s.h).

The library is the product: every pixel this package produces comes from its
HIP kernels.  There is no Python or CPU fallback for the pixel path — if the
shared object is missing or a GPU call fails, the error propagates.
"""
from __future__ import annotations

import ctypes
import math
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('H2S_LIB') or os.path.join(_HERE, 'libh2s.so')

# ---- error codes (include/h2s.h) ------------------------------------------
H2S_OK = 0
H2S_E_INVALID_ARG = -1
H2S_E_UNSUPPORTED = -2
H2S_E_HIP = -3
H2S_E_OOM = -4
H2S_E_LUT_MISSING = -5
H2S_E_PARSE = -6

TRC_PQ, TRC_HLG = 0, 1
TM_NONE, TM_LINEAR, TM_GAMMA, TM_CLIP, TM_REINHARD, TM_HABLE, TM_MOBIUS, TM_BT2390, TM_SPLINE = range(9)
MODE_COMPAT8, MODE_NATIVE = 0, 1
DESAT_LUMA_RGB, DESAT_LUMA_BT2020, DESAT_LUMA_BT709 = 0, 1, 2
LOC_DEVICE, LOC_HOST = 0, 1
STAGE_LINEAR, STAGE_TONEMAP, STAGE_GAMMA, STAGE_LUT, STAGE_YUV = 1, 2, 3, 4, 5
CHROMA_BOX, CHROMA_BICUBIC = 0, 1
DITHER_NONE, DITHER_ORDERED = 0, 1
EXPAND_SHIFT, EXPAND_REPLICATE = 0, 1
EDGE_ZIMG, EDGE_REPLICATE, EDGE_MIRROR = 0, 1, 2
LUT_IN_FLOAT, LUT_IN_RGB48 = 0, 1
LP_TONE_IPT, LP_TONE_MAX_RGB = 0, 1
LP_RANGE_FULL, LP_RANGE_LIMITED = 0, 1
LP_DITHER_NONE, LP_DITHER_ORDERED = 0, 1
LP_P010_KEEP, LP_P010_TRUNCATE = 0, 1
PIPE_AUTO, PIPE_CPU_CHAIN, PIPE_LIBPLACEBO = 0, 1, 2
OPT_FAST_PATH, OPT_TILES_PER_BLOCK, OPT_HOST_SERIAL, OPT_LP_EXACT = 1, 2, 3, 5
OPT_RESERVED_4 = 4   # H2S_OPT_LP_EXACT's key in ABI 3.3: now INVALID_ARG
# private test hook (include/h2s.h H2S_PRIVATE_TEST_HOOKS: not part of the ABI)
OPT_TEST_FAIL_AFTER_LAUNCH = 0x7f000000 + 1
OPT_TEST_PEAK_FORM = 0x7f000000 + 2
OPT_TEST_PEAK_CHUNK = 0x7f000000 + 3
OPT_TEST_PEAK_BLOCKS = 0x7f000000 + 4
PATH_TILE, PATH_TILE_TAIL, PATH_GENERIC, PATH_TWO_PASS = 1, 2, 3, 4
ABI_VERSION = 3
ABI_MINOR = 4   # include/h2s.h H2S_ABI_MINOR (the loaded library may be newer, not older)

# every symbol include/h2s.h declares (checked by tests/test_abi_exports.py)
EXPORTS = (
    'h2s_abi_version', 'h2s_abi_minor', 'h2s_create', 'h2s_destroy', 'h2s_last_error',
    'h2s_set_lut', 'h2s_params_default', 'h2s_set_params', 'h2s_process',
    'h2s_debug_float', 'h2s_cube_generate', 'h2s_cube_format', 'h2s_cube_parse',
    'h2s_kernel_ms', 'h2s_set_timing', 'h2s_preview_size', 'h2s_preview_rgb24', 'h2s_preview_rgb24_batch', 'h2s_peak_reset',
    'h2s_peak_state', 'h2s_peak_stats', 'h2s_peak_feed', 'h2s_set_option', 'h2s_query_path',
)


class H2SParams(ctypes.Structure):
    _fields_ = [
        ('transfer_in', ctypes.c_int32),
        ('bits_in', ctypes.c_int32),
        ('bits_out', ctypes.c_int32),
        ('tonemap', ctypes.c_int32),
        ('tm_param', ctypes.c_double),
        ('desat', ctypes.c_double),
        ('peak', ctypes.c_double),
        ('npl', ctypes.c_double),
        ('gamma', ctypes.c_double),
        ('maxcll', ctypes.c_double),
        ('mastering_max', ctypes.c_double),
        ('lut_enabled', ctypes.c_int32),
        ('mode', ctypes.c_int32),
        ('desat_luma', ctypes.c_int32),
        ('peak_detect', ctypes.c_int32),
        ('chroma_filter', ctypes.c_int32),
        ('dither', ctypes.c_int32),
        ('expand', ctypes.c_int32),
        ('pipeline', ctypes.c_int32),
        ('knee_offset', ctypes.c_double),
        ('target_black', ctypes.c_double),
        ('target_white', ctypes.c_double),
        ('chroma_edge', ctypes.c_int32),
        ('lut_input', ctypes.c_int32),
        ('lp_tone', ctypes.c_int32),
        # ABI v3: libplacebo branch options and peak_detect parameters
        ('lp_range', ctypes.c_int32), ('lp_dither', ctypes.c_int32), ('lp_p010', ctypes.c_int32),
        ('reserved', ctypes.c_int32 * 2),
        ('pd_smoothing', ctypes.c_double), ('pd_scene_low', ctypes.c_double),
        ('pd_scene_high', ctypes.c_double), ('pd_percentile', ctypes.c_double),
        ('pd_min_peak', ctypes.c_double),
    ]


class H2SFrames(ctypes.Structure):
    _fields_ = [
        ('data', ctypes.c_void_p * 3),
        ('linesize', ctypes.c_int64 * 3),
        ('frame_pitch', ctypes.c_int64 * 3),
        ('width', ctypes.c_int32),
        ('height', ctypes.c_int32),
        ('bits', ctypes.c_int32),
        ('location', ctypes.c_int32),
    ]


class H2SError(RuntimeError):
    """A libh2s call failed (HIP error, OOM, ...).  Subclasses RuntimeError:
    the reference surfaces a failed ffmpeg run as RuntimeError
    (src/utils.py:297-308)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f'libh2s error {code}: {msg}')
        self.code = code


def raise_for(code: int, msg: str) -> None:
    """Map an H2S_E_* code onto the reference's exception types."""
    if code == H2S_OK:
        return
    if code == H2S_E_LUT_MISSING:
        # src/utils.py:185-186: a missing bundled LUT is FileNotFoundError
        raise FileNotFoundError(msg)
    if code in (H2S_E_INVALID_ARG, H2S_E_UNSUPPORTED, H2S_E_PARSE):
        # src/ffmpeg_command.py:240-245: an impossible request is ValueError
        raise ValueError(msg)
    raise H2SError(code, msg)


_lib = None


def lib() -> ctypes.CDLL:
    """Load libh2s once.  Raises ImportError when the extension was not
    built — the pixel path has no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f'libh2s.so not found at {LIB_PATH}; build it with '
            '`python -c "import __graft_entry__ as g; g.build()"` (hipcc, gfx950)')
    # torch ships its own libamdhip64 with the same SONAME; importing torch
    # first makes libh2s bind to that single HIP runtime instead of loading a
    # second copy from /opt/rocm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    c_ctx = ctypes.c_void_p
    sig = {
        'h2s_abi_version': (ctypes.c_int, []),
        'h2s_abi_minor': (ctypes.c_int, []),
        'h2s_create': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_ctx)]),
        'h2s_destroy': (None, [c_ctx]),
        'h2s_last_error': (ctypes.c_char_p, [c_ctx]),
        'h2s_set_lut': (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_int]),
        'h2s_params_default': (None, [ctypes.POINTER(H2SParams)]),
        'h2s_set_params': (ctypes.c_int, [c_ctx, ctypes.POINTER(H2SParams)]),
        'h2s_process': (ctypes.c_int, [c_ctx, ctypes.POINTER(H2SFrames), ctypes.POINTER(H2SFrames),
                                       ctypes.c_int, ctypes.c_void_p]),
        'h2s_debug_float': (ctypes.c_int, [c_ctx, ctypes.POINTER(H2SFrames), ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
        'h2s_cube_generate': (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
        'h2s_cube_format': (ctypes.c_int64, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int64]),
        'h2s_cube_parse': (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]),
        'h2s_kernel_ms': (ctypes.c_double, [c_ctx, ctypes.c_int]),
        'h2s_set_timing': (ctypes.c_int, [c_ctx, ctypes.c_int]),
        'h2s_peak_reset': (ctypes.c_int, [c_ctx]),
        'h2s_peak_state': (ctypes.c_int, [c_ctx, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
        'h2s_peak_stats': (ctypes.c_int, [c_ctx, ctypes.POINTER(H2SFrames), ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]),
        'h2s_peak_feed': (ctypes.c_int, [c_ctx, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
        'h2s_set_option': (ctypes.c_int, [c_ctx, ctypes.c_int, ctypes.c_int64]),
        'h2s_query_path': (ctypes.c_int, [c_ctx, ctypes.POINTER(H2SFrames), ctypes.POINTER(H2SFrames)]),
        'h2s_preview_size': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
        'h2s_preview_rgb24': (ctypes.c_int, [c_ctx, ctypes.POINTER(H2SFrames), ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                             ctypes.c_void_p]),
        'h2s_preview_rgb24_batch': (ctypes.c_int, [c_ctx, ctypes.POINTER(H2SFrames), ctypes.c_int, ctypes.c_void_p,
                                                   ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_double, ctypes.c_int, ctypes.c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.h2s_abi_version() != ABI_VERSION:
        raise ImportError(f'libh2s ABI {L.h2s_abi_version()} != {ABI_VERSION}')
    if L.h2s_abi_minor() < ABI_MINOR:
        raise ImportError(f'libh2s ABI 3.{L.h2s_abi_minor()} is older than the 3.{ABI_MINOR} these bindings need')
    _lib = L
    return L


def default_params() -> H2SParams:
    p = H2SParams()
    lib().h2s_params_default(ctypes.byref(p))
    return p


NAN = math.nan
