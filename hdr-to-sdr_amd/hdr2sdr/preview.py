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

Which chain: the reference previews through libplacebo
(``extract_frame_with_gpu_conversion``, src/utils.py:768-800: its
``build_libplacebo_filter`` chain, so ``peak_detect=1`` and the LUT switch)
for the GPU-only operators and whenever GPU tone mapping is on
(``_use_gpu_extraction``, src/preview.py:584-590), and through
FFMPEG_FILTER otherwise, where ``lut_enabled=False`` selects
FFMPEG_FILTER_LEGACY_NO_LUT (src/utils.py:57-60).  ``convert_batch`` is the
batched form (``extract_frames_with_conversion_batch`` /
``extract_frames_with_gpu_conversion_batch``, src/utils.py:668-716, :803-824).
"""
from __future__ import annotations

import ctypes
import math
import re
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from . import lut as _lut
from .chain import TonemapParams, is_gpu_only_tonemapper, parse_filter_chain
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


def use_gpu_extraction(tonemapper: str, gpu_tonemap_active: bool = False) -> bool:
    """src/preview.py:584-590: the libplacebo preview for the GPU-only
    operators, and for every operator while GPU tone mapping is on."""
    return is_gpu_only_tonemapper(tonemapper) or bool(gpu_tonemap_active)


def preview_params(tonemapper: str, lut_enabled: bool = True, use_gpu: bool = False, bits_in: int = 10,
                   transfer: str = 'smpte2084', **params: Any) -> TonemapParams:
    """The chain the reference's preview runs (gamma 1.0, yuv420p / rgba8
    out): ``build_libplacebo_filter(1.0, tm, w, h, lut_enabled)`` — peak
    detection on, the plain-Vulkan ``format=p010,hwupload`` upload — or
    FFMPEG_FILTER (LUT always on) / FFMPEG_FILTER_LEGACY_NO_LUT."""
    tm = tonemapper.lower()
    kw: 'dict[str, Any]' = dict(tonemapper=tm, gamma=1.0, bits_in=bits_in, bits_out=8, transfer=transfer,
                                lut_enabled=lut_enabled)
    if use_gpu_extraction(tm, use_gpu):
        kw.update(pipeline='libplacebo', desat=0.0, peak_detect=True, lp_p010='truncate')
    else:
        kw.update(pipeline='cpu')
    kw.update(params)
    return TonemapParams(**kw)


def parse_preview_chain(chain: str, bits_in: int = 10, transfer: str = 'smpte2084',
                        **overrides: Any) -> 'tuple[TonemapParams, str | None, tuple[int | str, int | str]]':
    """A preview ``-vf`` string the reference builds -> (params, lut path, box).
    FFMPEG_FILTER / FFMPEG_FILTER_LEGACY_NO_LUT end in
    ``scale=W:H:force_original_aspect_ratio=decrease`` (src/utils.py:46-49,
    :57-60); the libplacebo preview carries the box as its ``w=`` / ``h=``
    (src/utils.py:787).  The box goes to ``Previewer.convert`` (an aspect
    fit for the CPU chain's ``scale=``, exactly the box for the libplacebo
    preview: ``Previewer.out_size``); the chain itself runs at the source size
    and bits_out 8, so the libplacebo stage's numeric ``w=`` / ``h=`` are
    replaced by ``iw`` / ``ih`` before ``parse_filter_chain``, which accepts
    only those for a conversion chain."""
    box: 'tuple[int | str, int | str]' = ('iw', 'ih')
    parts = chain.rsplit(',', 1)
    if len(parts) == 2 and parts[1].startswith('scale='):
        opts = parts[1][len('scale='):].split(':')
        kv = dict(o.split('=', 1) for o in opts[2:] if '=' in o)
        if len(opts) < 2 or kv.get('force_original_aspect_ratio', 'decrease') != 'decrease':
            raise ValueError(f'preview scale stage {parts[1]!r} is not the reference\'s aspect-fit box')
        box = tuple(v if v in ('iw', 'ih') else int(v) for v in opts[:2])   # type: ignore[assignment]
        chain = parts[0]
    else:
        m = re.search(r'libplacebo=w=(\w+):h=(\w+)', chain)
        if m:
            for v in m.groups():
                if v not in ('iw', 'ih') and not (v.isdigit() and int(v) > 0):
                    raise ValueError(f'libplacebo preview size {v!r} is not modelled (iw / ih or a positive integer)')
            box = tuple(v if v in ('iw', 'ih') else int(v) for v in m.groups())   # type: ignore[assignment]
            chain = chain[:m.start()] + 'libplacebo=w=iw:h=ih' + chain[m.end():]
    params, lut = parse_filter_chain(chain, bits_in=bits_in, bits_out=8, transfer=transfer, **overrides)
    return params, lut, box


class Previewer:
    """One libh2s context configured for previews. The chain runs at
    bits_out 8 with eq gamma 1.0, as extract_frame_with_conversion(gamma=1.0)
    and extract_frame_with_gpu_conversion(gamma=1.0) do. ``use_gpu``: GPU
    tone mapping is on (the GUI's toggle, src/preview.py:570-582), which
    selects the libplacebo preview for every operator; the GPU-only
    operators take it regardless.  ``lut_enabled=False`` is
    FFMPEG_FILTER_LEGACY_NO_LUT's closed-form gamut path on the CPU chain
    (src/utils.py:57-60) and libplacebo's own BT.709 conversion on the GPU
    one.  Each preview frame starts from a fresh peak state, as each of the
    reference's preview ffmpeg runs does."""

    def __init__(self, device: int = 0, tonemapper: str = 'reinhard', lut_enabled: bool = True,
                 bits_in: int = 10, transfer: str = 'smpte2084', lattice: Optional[np.ndarray] = None,
                 use_gpu: bool = False, params: Optional[TonemapParams] = None, **kw: Any):
        from .engine import Tonemapper
        if params is None:
            params = preview_params(tonemapper, lut_enabled, use_gpu, bits_in, transfer, **kw)
        elif params.bits_out != 8 or params.gamma != 1.0:
            raise ValueError('a preview chain runs at bits_out 8 and gamma 1.0 (the display gamma is separate)')
        self.params = params
        lut_enabled = params.lut_enabled
        self._tm = Tonemapper(device, self.params)
        if lut_enabled:
            self._tm.set_lut(lattice if lattice is not None else _lut.generate_lattice(_lut.LUT_SIZE))

    @classmethod
    def from_chain(cls, chain: str, device: int = 0, bits_in: int = 10, transfer: str = 'smpte2084',
                   lattice: Optional[np.ndarray] = None) -> 'tuple[Previewer, tuple[int | str, int | str]]':
        """A Previewer for a reference preview ``-vf`` string, and its box."""
        params, _, box = parse_preview_chain(chain, bits_in=bits_in, transfer=transfer)
        return cls(device, lattice=lattice, params=params), box

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
        return self._run(frame.slice(0, 1) if frame.nframes > 1 else frame, width, height, gamma)[0]

    def convert_batch(self, frames: 'FrameBatch | Sequence[FrameBatch]', width: 'int | str' = PREVIEW_SIZE[0],
                      height: 'int | str' = PREVIEW_SIZE[1], gamma: float = 1.0) -> List[np.ndarray]:
        """RGB24 previews of several frames: every frame of one FrameBatch, or
        frame 0 of each batch in a list (frames of different sizes allowed).
        Frames of one size run as one libh2s call (one tone-map launch on the
        CPU chain; one resize and one RGB launch per plane either way)."""
        if isinstance(frames, FrameBatch):
            return self._run(frames, width, height, gamma)
        out: 'list[np.ndarray | None]' = [None] * len(frames)
        groups: 'dict[tuple[int, int, int, bool, Any], list[int]]' = {}
        for i, f in enumerate(frames):
            key = (f.width, f.height, f.bits, f.is_torch, getattr(f.buf, 'device', None))
            groups.setdefault(key, []).append(i)
        for idx in groups.values():
            firsts = [frames[i] if frames[i].nframes == 1 else frames[i].slice(0, 1) for i in idx]
            if firsts[0].is_torch:
                import torch
                buf = torch.cat([f.buf for f in firsts])
            else:
                buf = np.concatenate([np.asarray(f.buf) for f in firsts])
            batch = FrameBatch(buf, firsts[0].width, firsts[0].height, firsts[0].bits)
            for i, img in zip(idx, self._run(batch, width, height, gamma)):
                out[i] = img
        return out   # type: ignore[return-value]

    def out_size(self, in_w: int, in_h: int, width: 'int | str' = PREVIEW_SIZE[0],
                 height: 'int | str' = PREVIEW_SIZE[1]) -> Tuple[int, int]:
        """The preview's output size for an in_w x in_h frame and the box.
        CPU chain: FFMPEG_FILTER's ``scale=W:H:force_original_aspect_ratio=decrease``
        (src/utils.py:46-49), an aspect fit.  libplacebo preview:
        ``build_libplacebo_filter`` passes ``w=W:h=H`` with no aspect option
        (src/utils.py:446, :787), and vf_libplacebo's own default
        (force_original_aspect_ratio disabled) outputs exactly W x H, so a
        non-16:9 source is stretched to the box as the reference does (the
        resampling filter libplacebo uses for it is not restated: PARITY
        UNPINNED; the swscale-style bicubic of the CPU preview is used)."""
        bw = in_w if width == 'iw' else int(width)
        bh = in_h if height == 'ih' else int(height)
        if self.params.resolved_pipeline() == 'libplacebo':
            if bw <= 0 or bh <= 0:
                raise ValueError(f'preview box must be positive, got {bw}x{bh}')
            return bw, bh
        return fit_size(in_w, in_h, bw, bh)

    def _run(self, frames: FrameBatch, width: 'int | str', height: 'int | str', gamma: float) -> List[np.ndarray]:
        ow, oh = self.out_size(frames.width, frames.height, width, height)
        n = frames.nframes
        out = np.empty((n, oh, ow, 3), dtype=np.uint8)
        d = frames.descriptor()
        L = _abi.lib()
        rc = L.h2s_preview_rgb24_batch(self._tm._ctx, ctypes.byref(d), n, out.ctypes.data, 3 * ow, 3 * ow * oh,
                                       ow, oh, float(gamma), _abi.LOC_HOST, self._tm._stream_ptr(None))
        if rc:
            _abi.raise_for(rc, L.h2s_last_error(self._tm._ctx).decode())
        return [out[i] for i in range(n)]
