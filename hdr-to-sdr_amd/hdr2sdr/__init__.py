"""hdr2sdr — MI355X-native HDR10/HLG -> SDR tone mapping.

Drop-in replacement for the CPU ffmpeg filter chain of TORlN/HDR-to-SDR
(src/utils.py:38-42), executed by hand-written HIP kernels for gfx950 through
the C-ABI library libh2s (include/h2s.h).
"""
from ._abi import H2SError, lib  # noqa: F401
from .chain import (FFMPEG_CONVERT_FILTER, GPU_ONLY_TONEMAPPERS, TONEMAP,  # noqa: F401
                    TonemapParams, is_gpu_only_tonemapper, parse_filter_chain)
from .engine import Tonemapper  # noqa: F401
from .frames import FrameBatch, frame_bytes  # noqa: F401
from .lut import LUT_SIZE, cube_text, generate_cube_lines, generate_lattice, load_cube, parse_cube  # noqa: F401
from .plan import H2SProcess, PipePlan, plan_from_argv  # noqa: F401
from .preview import PREVIEW_SIZE, Previewer, fit_size  # noqa: F401

__all__ = [
    'FFMPEG_CONVERT_FILTER', 'GPU_ONLY_TONEMAPPERS', 'TONEMAP', 'TonemapParams',
    'is_gpu_only_tonemapper', 'parse_filter_chain', 'Tonemapper', 'FrameBatch',
    'frame_bytes', 'LUT_SIZE', 'cube_text', 'generate_cube_lines', 'generate_lattice',
    'load_cube', 'parse_cube', 'H2SError', 'lib', 'H2SProcess', 'PipePlan', 'plan_from_argv',
    'PREVIEW_SIZE', 'Previewer', 'fit_size',
]
