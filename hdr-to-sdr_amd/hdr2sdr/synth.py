"""Seeded synthetic HDR10 / HLG frames (SURVEY.md §8d input distributions).

The reference's pixel fixtures (test/smoke_test_videos/*.mp4) are HEVC and
cannot be decoded without ffmpeg, so parity tests and the benchmark use
synthetic planar frames of the same shape:

* ``uniform`` — every sample uniform over the legal limited range
  (10-bit: Y 64..940, C 64..960; 12-bit: x4).  Worst case for the 3D-LUT
  gathers (no locality).
* ``smooth``  — low-frequency value noise in PQ/HLG R'G'B', converted to
  BT.2020-NCL limited-range Y'CbCr (realistic locality; bench headline).
* ``ramp``    — PQ code 0..1 along x (0..10000 nits), hue sweep along y.
* ``edges``   — out-of-range and extreme codes (0..63, 941..1023, chroma
  extremes) mixed at random: exercises clamps, negatives and NaN guards.

Generation runs in torch on whatever device the caller names, seeded per
frame from ``seed + frame_index``.

``frames_from_rgb8`` turns a captured frame (8-bit R'G'B' read as PQ BT.2020
codes, e.g. the reference's own website HDR frame, tests/golden/) into the
same planar layout: real content between ``smooth`` and ``uniform``.
"""
from __future__ import annotations

from typing import Any

from .frames import FrameBatch

KINDS = ('uniform', 'smooth', 'ramp', 'edges')


def _gen(seed: int, device: Any):
    import torch
    g = torch.Generator(device='cpu')
    g.manual_seed(seed)
    return g


def _rgb_to_frame(rgb, bits: int):
    """R'G'B' in [0,1] float [3,H,W] -> (Y, U, V) int tensors, BT.2020-NCL,
    limited range, 2x2-averaged chroma."""
    import torch
    kr, kb = 0.2627, 0.0593
    kg = 1 - kr - kb
    r, g, b = rgb[0], rgb[1], rgb[2]
    y = kr * r + kg * g + kb * b
    cb = (b - y) / (2 * (1 - kb))
    cr = (r - y) / (2 * (1 - kr))
    s = float(1 << (bits - 8))
    hi = (1 << bits) - 1
    Y = torch.clamp(torch.round((16 + 219 * y) * s), 0, hi)

    def sub(c):
        h, w = c.shape
        c = c.reshape(h // 2, 2, w // 2, 2).mean(dim=(1, 3))
        return torch.clamp(torch.round((128 + 224 * c) * s), 0, hi)
    return Y, sub(cb), sub(cr)


def synth_frames(kind: str, nframes: int, width: int, height: int, bits: int = 10,
                 device: Any = 'cpu', seed: int = 0x5EED) -> FrameBatch:
    import torch
    if kind not in KINDS:
        raise ValueError(f'unknown synthetic kind {kind!r}; expected one of {KINDS}')
    fb = FrameBatch.empty_torch(nframes, width, height, bits, device)
    s = 1 << (bits - 8)
    for i in range(nframes):
        g = _gen(seed + i, device)
        if kind == 'uniform':
            fb.y[i] = torch.randint(16 * s, 235 * s + 1, (height, width), generator=g).to(fb.buf.dtype).to(device)
            fb.u[i] = torch.randint(16 * s, 240 * s + 1, (height // 2, width // 2), generator=g).to(fb.buf.dtype).to(device)
            fb.v[i] = torch.randint(16 * s, 240 * s + 1, (height // 2, width // 2), generator=g).to(fb.buf.dtype).to(device)
            continue
        if kind == 'edges':
            hi = (1 << bits) - 1

            def pick(shape):
                lo_band = torch.randint(0, 16 * s, shape, generator=g)
                hi_band = torch.randint(235 * s, hi + 1, shape, generator=g)
                mid = torch.randint(16 * s, 240 * s + 1, shape, generator=g)
                sel = torch.randint(0, 3, shape, generator=g)
                return torch.where(sel == 0, lo_band, torch.where(sel == 1, hi_band, mid))
            fb.y[i] = pick((height, width)).to(fb.buf.dtype).to(device)
            fb.u[i] = pick((height // 2, width // 2)).to(fb.buf.dtype).to(device)
            fb.v[i] = pick((height // 2, width // 2)).to(fb.buf.dtype).to(device)
            continue
        if kind == 'smooth':
            gh, gw = max(2, height // 120 + 2), max(2, width // 120 + 2)
            grid = torch.rand((1, 3, gh, gw), generator=g).to(device)
            grid = 0.05 + 0.9 * grid
            rgb = torch.nn.functional.interpolate(grid, size=(height, width), mode='bicubic',
                                                  align_corners=True)[0].clamp(0, 1)
        else:  # ramp
            xs = torch.linspace(0, 1, width, device=device)
            ys = torch.linspace(0, 1, height, device=device)
            hue = ys[:, None] * 6.0
            base = xs[None, :].expand(height, width)
            r = base * torch.clamp(torch.abs(hue - 3) - 1, 0, 1)
            gg = base * torch.clamp(2 - torch.abs(hue - 2), 0, 1)
            b = base * torch.clamp(2 - torch.abs(hue - 4), 0, 1)
            # keep a neutral band in the top rows (pure grey ramp)
            neutral = (ys[:, None] < 0.1).expand(height, width)
            rgb = torch.stack([torch.where(neutral, base, r), torch.where(neutral, base, gg),
                               torch.where(neutral, base, b)])
        Y, U, V = _rgb_to_frame(rgb.float(), bits)
        fb.y[i] = Y.to(fb.buf.dtype)
        fb.u[i] = U.to(fb.buf.dtype)
        fb.v[i] = V.to(fb.buf.dtype)
    return fb


def frames_from_rgb8(rgb8: Any, nframes: int, bits: int = 10, device: Any = 'cpu') -> FrameBatch:
    """uint8 [H, W, 3] R'G'B' (PQ BT.2020 codes / 255) -> ``nframes`` copies
    as BT.2020-NCL limited-range Y'CbCr 4:2:0 (H and W cropped to even)."""
    import torch
    t = torch.as_tensor(rgb8)
    h, w = t.shape[0] & ~1, t.shape[1] & ~1
    rgb = t[:h, :w].permute(2, 0, 1).to(device=device, dtype=torch.float32) / 255.0
    Y, U, V = _rgb_to_frame(rgb, bits)
    fb = FrameBatch.empty_torch(nframes, w, h, bits, device)
    for i in range(nframes):
        fb.y[i], fb.u[i], fb.v[i] = Y.to(fb.buf.dtype), U.to(fb.buf.dtype), V.to(fb.buf.dtype)
    return fb
