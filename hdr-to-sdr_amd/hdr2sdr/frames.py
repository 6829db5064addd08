"""Planar 4:2:0 frame batches (yuv420p / yuv420p10le / yuv420p12le).

The reference never holds frames itself: ffmpeg owns every buffer
(SURVEY.md §8b "Ownership").  Here the caller owns them, in device memory
(torch tensors on a HIP device) or host memory (numpy), and describes them to
libh2s with an ``h2s_frames`` record: one base pointer, linesize and
frame pitch per plane.

Layout in HBM: one contiguous allocation per batch, frames back to back, each
frame = Y plane (H x W) then U (H/2 x W/2) then V, rows packed (linesize =
width * bytes-per-sample).  A 3840x2160 10-bit frame is 24,883,200 B, so a
288 GB MI355X holds >10,000 such frames; batches of 16-64 frames per launch
keep the grid far above the 256-CU fill point.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Any

import numpy as np

from . import _abi


def sample_bytes(bits: int) -> int:
    return 1 if bits == 8 else 2


def frame_bytes(width: int, height: int, bits: int) -> int:
    return width * height * sample_bytes(bits) * 3 // 2


@dataclass
class FrameBatch:
    """``nframes`` planar 4:2:0 frames in one contiguous buffer.

    ``buf`` is a 2-D array/tensor [nframes, frame_bytes/sample_bytes] of
    uint8 (8-bit) or int16 (10/12-bit samples stored little-endian in 16
    bits, the *le formats).  Plane views are exposed as y / u / v."""
    buf: Any
    width: int
    height: int
    bits: int

    # ---- constructors ---------------------------------------------------
    @staticmethod
    def _shape(nframes: int, width: int, height: int, bits: int) -> 'tuple[int, int]':
        if width <= 0 or height <= 0 or width % 2 or height % 2:
            raise ValueError(f'4:2:0 frames need positive even dimensions, got {width}x{height}')
        if bits not in (8, 10, 12):
            raise ValueError(f'bits must be 8, 10 or 12, got {bits}')
        return nframes, width * height * 3 // 2

    @classmethod
    def empty_torch(cls, nframes: int, width: int, height: int, bits: int, device: Any) -> 'FrameBatch':
        import torch
        dt = torch.uint8 if bits == 8 else torch.int16
        return cls(torch.empty(cls._shape(nframes, width, height, bits), dtype=dt, device=device),
                   width, height, bits)

    @classmethod
    def empty_numpy(cls, nframes: int, width: int, height: int, bits: int) -> 'FrameBatch':
        dt = np.uint8 if bits == 8 else np.uint16
        return cls(np.zeros(cls._shape(nframes, width, height, bits), dtype=dt), width, height, bits)

    @classmethod
    def empty_pinned(cls, nframes: int, width: int, height: int, bits: int) -> 'FrameBatch':
        """Host batch in page-locked memory (DMA-able without a bounce copy:
        the host-buffer path of h2s_process then runs at PCIe speed). Falls
        back to pageable numpy memory when no GPU runtime is present."""
        try:
            import torch
            if torch.cuda.is_available():
                dt = torch.uint8 if bits == 8 else torch.int16
                t = torch.empty(cls._shape(nframes, width, height, bits), dtype=dt, pin_memory=True)
                a = t.numpy() if bits == 8 else t.numpy().view(np.uint16)
                fb = cls(a, width, height, bits)
                fb._pin = t          # keep the pinned allocation alive
                return fb
        except (ImportError, RuntimeError):
            pass
        return cls.empty_numpy(nframes, width, height, bits)

    @classmethod
    def from_planes(cls, y: np.ndarray, u: np.ndarray, v: np.ndarray, bits: int) -> 'FrameBatch':
        """Pack [F,H,W] / [F,H/2,W/2] numpy planes into a batch."""
        f, h, w = y.shape
        fb = cls.empty_numpy(f, w, h, bits)
        fb.y[...] = y
        fb.u[...] = u
        fb.v[...] = v
        return fb

    # ---- plane views ------------------------------------------------------
    @property
    def nframes(self) -> int:
        return int(self.buf.shape[0])

    @property
    def is_torch(self) -> bool:
        return not isinstance(self.buf, np.ndarray)

    def _plane(self, p: int):
        w, h = self.width, self.height
        ysz = w * h
        csz = ysz // 4
        if p == 0:
            return self.buf[:, :ysz].reshape(self.nframes, h, w)
        off = ysz + (p - 1) * csz
        return self.buf[:, off:off + csz].reshape(self.nframes, h // 2, w // 2)

    @property
    def y(self):
        return self._plane(0)

    @property
    def u(self):
        return self._plane(1)

    @property
    def v(self):
        return self._plane(2)

    def to_numpy(self) -> 'FrameBatch':
        if not self.is_torch:
            return self
        a = self.buf.detach().cpu().numpy()
        if self.bits != 8:
            a = a.view(np.uint16)
        return FrameBatch(a, self.width, self.height, self.bits)

    def to_torch(self, device: Any) -> 'FrameBatch':
        import torch
        if self.is_torch:
            return FrameBatch(self.buf.to(device), self.width, self.height, self.bits)
        a = self.buf if self.bits == 8 else self.buf.view(np.int16)
        return FrameBatch(torch.from_numpy(np.ascontiguousarray(a)).to(device), self.width, self.height, self.bits)

    def slice(self, start: int, stop: int) -> 'FrameBatch':
        return FrameBatch(self.buf[start:stop], self.width, self.height, self.bits)

    # ---- C-ABI descriptor ---------------------------------------------------
    def descriptor(self) -> _abi.H2SFrames:
        d = _abi.H2SFrames()
        sb = sample_bytes(self.bits)
        w, h = self.width, self.height
        if self.is_torch:
            if not self.buf.is_contiguous():
                raise ValueError('frame buffer must be contiguous')
            base = self.buf.data_ptr()
            loc = _abi.LOC_DEVICE if self.buf.is_cuda else _abi.LOC_HOST
        else:
            if not self.buf.flags['C_CONTIGUOUS']:
                raise ValueError('frame buffer must be C-contiguous')
            base = self.buf.ctypes.data
            loc = _abi.LOC_HOST
        ysz = w * h * sb
        csz = ysz // 4
        fpitch = ysz + 2 * csz
        d.data[0] = base
        d.data[1] = base + ysz
        d.data[2] = base + ysz + csz
        d.linesize[0] = w * sb
        d.linesize[1] = d.linesize[2] = (w // 2) * sb
        for p in range(3):
            d.frame_pitch[p] = fpitch
        d.width, d.height, d.bits, d.location = w, h, self.bits, loc
        return d


def descriptor_ptr(fb: FrameBatch):
    d = fb.descriptor()
    return d, ctypes.byref(d)
