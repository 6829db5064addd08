"""Tonemapper: one libh2s context on one GPU.

Replaces what the reference does per conversion — spawn ffmpeg with the chain
(src/conversion.py:209-224) and let it run filter_frame per frame — with a
context that holds the LUT lattice and resolved parameters in HBM and launches
the fused HIP kernel over whole batches of device-resident frames.
"""
from __future__ import annotations

import ctypes
from typing import Any

import numpy as np

from . import _abi
from .chain import TonemapParams, parse_filter_chain
from .frames import FrameBatch
from . import lut as _lut


class Tonemapper:
    """One context per GPU / worker (contexts share no state)."""

    def __init__(self, device: int = 0, params: 'TonemapParams | None' = None,
                 lut: 'np.ndarray | None' = None):
        L = _abi.lib()
        self._L = L
        ctx = ctypes.c_void_p()
        rc = L.h2s_create(int(device), ctypes.byref(ctx))
        if rc != 0:
            _abi.raise_for(rc, L.h2s_last_error(None).decode())
        self._ctx = ctx
        self.device = device
        self.params: 'TonemapParams | None' = None
        self.lut_size = 0
        if params is not None:
            self.set_params(params)
        if lut is not None:
            self.set_lut(lut)

    # ---- lifecycle --------------------------------------------------------
    def close(self) -> None:
        if getattr(self, '_ctx', None) and self._ctx.value:
            self._L.h2s_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self) -> 'Tonemapper':
        return self

    def __exit__(self, *exc: Any) -> None:
        self.close()

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        if rc != 0:
            _abi.raise_for(rc, self._L.h2s_last_error(self._ctx).decode())

    # ---- configuration ------------------------------------------------------
    def set_params(self, params: TonemapParams) -> None:
        c = params.to_c()
        self._check(self._L.h2s_set_params(self._ctx, ctypes.byref(c)))
        self.params = params

    def set_lut(self, lattice: Any) -> None:
        """lattice: float32 [n^3, 3] (.cube order) as numpy, or a torch
        tensor (copied to host first)."""
        if not isinstance(lattice, np.ndarray):
            lattice = lattice.detach().cpu().numpy()
        a = np.ascontiguousarray(lattice, dtype=np.float32).reshape(-1, 3)
        n = round(a.shape[0] ** (1 / 3))
        if n ** 3 != a.shape[0]:
            raise ValueError(f'LUT has {a.shape[0]} entries, not a cube')
        self._check(self._L.h2s_set_lut(self._ctx, a.ctypes.data, n))
        self.lut_size = n

    def load_cube(self, path: str) -> None:
        self.set_lut(_lut.load_cube(path))

    def configure_from_chain(self, chain: str, **kw: Any) -> TonemapParams:
        """Drop-in: configure from a reference chain string (src/utils.py:38-42)."""
        params, path = parse_filter_chain(chain, **kw)
        self.set_params(params)
        if params.lut_enabled:
            if path is None or path == '<LUT>':
                self.set_lut(_lut.generate_lattice(_lut.LUT_SIZE))
            else:
                self.load_cube(_lut.unescape_filter_path(path))
        return params

    # ---- execution ----------------------------------------------------------
    @staticmethod
    def _stream_ptr(stream: Any) -> 'int | None':
        if stream is None:
            try:
                import torch
                if torch.cuda.is_available():
                    return torch.cuda.current_stream().cuda_stream
            except ImportError:
                pass
            return None
        return getattr(stream, 'cuda_stream', stream)

    def process(self, src: FrameBatch, dst: FrameBatch, stream: Any = None,
                nframes: 'int | None' = None) -> None:
        """Tone-map src into dst (asynchronous when both are on the device)."""
        n = src.nframes if nframes is None else nframes
        if n > src.nframes or n > dst.nframes:
            raise ValueError(f'nframes {n} exceeds the batch ({src.nframes} in, {dst.nframes} out)')
        di, do = src.descriptor(), dst.descriptor()
        self._check(self._L.h2s_process(self._ctx, ctypes.byref(di), ctypes.byref(do), int(n),
                                        self._stream_ptr(stream)))

    def __call__(self, src: FrameBatch, stream: Any = None) -> FrameBatch:
        if self.params is None:
            raise ValueError('set_params first')
        if src.is_torch:
            dst = FrameBatch.empty_torch(src.nframes, src.width, src.height, self.params.bits_out,
                                         src.buf.device)
        else:
            dst = FrameBatch.empty_numpy(src.nframes, src.width, src.height, self.params.bits_out)
        self.process(src, dst, stream)
        return dst

    def set_option(self, key: int, value: int) -> None:
        """h2s_set_option (_abi.OPT_FAST_PATH / OPT_TILES_PER_BLOCK / OPT_HOST_SERIAL / OPT_LP_EXACT)."""
        self._check(self._L.h2s_set_option(self._ctx, int(key), int(value)))

    def query_path(self, src: FrameBatch, dst: FrameBatch) -> int:
        """The kernel path (_abi.PATH_*) h2s_process would take for src -> dst."""
        di, do = src.descriptor(), dst.descriptor()
        rc = self._L.h2s_query_path(self._ctx, ctypes.byref(di), ctypes.byref(do))
        if rc < 0:
            self._check(rc)
        return rc

    def debug_float(self, src: FrameBatch, stage: int) -> np.ndarray:
        """float32 [3, H, W] of frame 0 after ``stage``: R, G, B for 1..4,
        the quantiser inputs (Y code, Cb, Cr in code units) for 5; computed by
        the kernel h2s_process would use (the tile kernel's debug instance on
        the tile path)."""
        out = np.empty((3, src.height, src.width), dtype=np.float32)
        d = src.descriptor()
        self._check(self._L.h2s_debug_float(self._ctx, ctypes.byref(d), int(stage), out.ctypes.data,
                                            _abi.LOC_HOST, self._stream_ptr(None)))
        return out

    # ---- dynamic peak (BT.2390 peak_detect) ----------------------------------
    def reset_peak(self) -> None:
        """Start a new sequence: forget the smoothed peak state."""
        self._check(self._L.h2s_peak_reset(self._ctx))

    def peak_stats(self, src: FrameBatch, stream: Any = None) -> 'tuple[np.ndarray, np.ndarray]':
        """Per-frame (max, mean) of PQ(max R,G,B) of a device batch: the
        statistics process() folds into the smoothing (h2s_peak_stats)."""
        n = src.nframes
        fmax, favg = np.zeros(n), np.zeros(n)
        di = src.descriptor()
        self._check(self._L.h2s_peak_stats(self._ctx, ctypes.byref(di), n, fmax.ctypes.data, favg.ctypes.data,
                                           self._stream_ptr(stream)))
        return fmax, favg

    def feed_peak(self, fmax: Any, favg: Any) -> None:
        """Fold frames' statistics into the smoothing state in order, without
        converting them (h2s_peak_feed): a frame-sharded rank replays the
        frames before its range."""
        fmax = np.ascontiguousarray(fmax, dtype=np.float64)
        favg = np.ascontiguousarray(favg, dtype=np.float64)
        if fmax.shape != favg.shape or fmax.ndim != 1:
            raise ValueError('fmax and favg must be 1-D arrays of one length')
        self._check(self._L.h2s_peak_feed(self._ctx, fmax.ctypes.data, favg.ctypes.data, int(fmax.size)))

    def peak_state(self) -> 'dict[str, float]':
        mx, avg, pk = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_int64()
        self._check(self._L.h2s_peak_state(self._ctx, ctypes.byref(mx), ctypes.byref(avg), ctypes.byref(pk),
                                           ctypes.byref(n)))
        return {'max_pq': mx.value, 'avg_pq': avg.value, 'peak': pk.value, 'frames': n.value}

    # ---- timing (bench) -----------------------------------------------------
    def set_timing(self, enabled: bool) -> None:
        self._check(self._L.h2s_set_timing(self._ctx, 1 if enabled else 0))

    def kernel_ms(self, count: int) -> float:
        return float(self._L.h2s_kernel_ms(self._ctx, int(count)))
