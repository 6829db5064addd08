"""Preview path.

The reference previews a frame with ``extract_frame_with_conversion``
(src/utils.py:719-765). That function runs FFMPEG_FILTER, which is the export
chain plus ``scale=W:H:force_original_aspect_ratio=decrease`` with the box
PREVIEW_SIZE = 3840x2160 (src/utils.py:46-49, src/preview.py:29). It always
runs the chain with gamma 1.0 and lets ffmpeg's PNG encoder convert
yuv420p -> rgb24. The GUI then applies ``adjust_gamma`` on R, G, B with
PIL's ``point()`` (src/preview.py:108-117).

Here all of that is one libh2s call per frame: the chain through k_tile,
the aspect-fit resize, the Y'CbCr -> RGB24 conversion and the display gamma,
run on the GPU, with the RGB returned as an ``(h, w, 3)`` uint8 array.
``PIL.Image.fromarray`` takes that array directly.
"""
from __future__ import annotations

import ctypes
import math
from typing import Any, Optional, Tuple

import numpy as np

from . import _abi
from . import lut as _lut
from .chain import TonemapParams
from .frames import FrameBatch

PREVIEW_SIZE = (3840, 2160)   # src/preview.py:29


def fit_size(in_w: int, in_h: int, box_w: int = PREVIEW_SIZE[0], box_h: int = PREVIEW_SIZE[1]) -> Tuple[int, int]:
    """Output size of ``scale=box_w:box_h:force_original_aspect_ratio=decrease``
    for an in_w x in_h frame (libavfilter scale_eval: av_rescale, then min
    with the box; the frame is upscaled when it is smaller than the box)."""
    w, h = ctypes.c_int(), ctypes.c_int()
    rc = _abi.lib().h2s_preview_size(int(in_w), int(in_h), int(box_w), int(box_h), ctypes.byref(w), ctypes.byref(h))
    if rc:
        _abi.raise_for(rc, _abi.lib().h2s_last_error(None).decode())
    return w.value, h.value


def adjust_gamma_lut(gamma: float) -> np.ndarray:
    """The 256-entry table the GUI's adjust_gamma passes to PIL's point()
    (src/preview.py:108-117), which the preview kernel applies."""
    if abs(gamma - 1.0) < 1e-6:
        return np.arange(256, dtype=np.uint8)
    inv = 1.0 / gamma
    return np.array([int(round(math.pow(i / 255.0, inv) * 255)) for i in range(256)], dtype=np.uint8)


class Previewer:
    """One libh2s context configured for previews. The chain runs at
    bits_out 8 with eq gamma 1.0, as extract_frame_with_conversion(gamma=1.0)
    does. ``lut_enabled=False`` is the reference's FFMPEG_FILTER_LEGACY_NO_LUT
    closed-form gamut path (src/utils.py:57-60)."""

    def __init__(self, device: int = 0, tonemapper: str = 'reinhard', lut_enabled: bool = True,
                 bits_in: int = 10, transfer: str = 'smpte2084', lattice: Optional[np.ndarray] = None,
                 **params: Any):
        from .engine import Tonemapper
        self.params = TonemapParams(tonemapper=tonemapper, gamma=1.0, bits_in=bits_in, bits_out=8,
                                    transfer=transfer, lut_enabled=lut_enabled, **params)
        self._tm = Tonemapper(device, self.params)
        if lut_enabled:
            self._tm.set_lut(lattice if lattice is not None else _lut.generate_lattice(_lut.LUT_SIZE))

    def close(self) -> None:
        self._tm.close()

    def __enter__(self) -> 'Previewer':
        return self

    def __exit__(self, *exc: Any) -> None:
        self.close()

    def convert(self, frame: FrameBatch, width: 'int | str' = PREVIEW_SIZE[0], height: 'int | str' = PREVIEW_SIZE[1],
                gamma: float = 1.0) -> np.ndarray:
        """RGB24 preview of frame 0 of ``frame`` (host or device batch). width /
        height: the box (``'iw'``/``'ih'`` keep the source size, as in the
        reference's defaults). gamma: the GUI's display gamma, fused here."""
        bw = frame.width if width == 'iw' else int(width)
        bh = frame.height if height == 'ih' else int(height)
        ow, oh = fit_size(frame.width, frame.height, bw, bh)
        out = np.empty((oh, ow, 3), dtype=np.uint8)
        d = frame.descriptor()
        L = _abi.lib()
        rc = L.h2s_preview_rgb24(self._tm._ctx, ctypes.byref(d), out.ctypes.data, 3 * ow, ow, oh, float(gamma),
                                 _abi.LOC_HOST, self._tm._stream_ptr(None))
        if rc:
            _abi.raise_for(rc, L.h2s_last_error(self._tm._ctx).decode())
        return out
