"""Gather locality of lane -> pixel geometries for the tile kernel's lattice
lookups (is a register-resident layout affordable?).
For each geometry, the 64 pixels one wave-wide gather covers are enumerated
over a 4K frame; per gather instruction (one of the 4 tetrahedral corners) the
distinct 64-B lines of the 12-B Y'CbCr-record lattice are counted.  Lattice
coordinates come from the oracle's stage-3 output (C2 params).  Test
infrastructure only (imports the oracle)."""
import sys
import numpy as np
sys.path.insert(0, 'hdr-to-sdr_amd')
sys.path.insert(0, '.')
import oracle
import hdr2sdr
from hdr2sdr.synth import synth_frames, frames_from_rgb8

N = 65
W, H = 3840, 2160


def coords(kind):
    p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
    if kind == 'real':
        rgb8 = np.load('tests/golden/website_hdr_full.npz')['hdr']
        fb = frames_from_rgb8(rgb8, 1, 10, 'cpu').to_numpy()
    else:
        fb = synth_frames(kind, 1, W, H, 10, device='cpu', seed=11).to_numpy()
    g = np.linspace(0, 1, N, dtype=np.float32)
    lat = np.stack(np.meshgrid(g, g, g, indexing="ij")[::-1], -1).reshape(-1, 3)   # any lattice: stage 3 is its input
    s = oracle.debug_float(oracle.params_from(p.to_c()), lat, fb.buf, W, H, 3) * (N - 1)
    return np.clip(s, 0, N - 1 - 1e-4)


def corner_offsets(s):
    i = np.floor(s).astype(np.int64)
    d = s - i
    order = np.argsort(-d, axis=0)
    E = np.eye(3, dtype=np.int64)[:, :, None, None]
    e0 = np.take_along_axis(np.broadcast_to(np.eye(3, dtype=np.int64)[:, :, None, None], (3, 3) + s.shape[1:]), order[None, :1], 1)[:, 0]
    e1 = np.take_along_axis(np.broadcast_to(np.eye(3, dtype=np.int64)[:, :, None, None], (3, 3) + s.shape[1:]), order[None, 1:2], 1)[:, 0]
    c = [i, i + e0, i + e0 + e1, i + 1]
    return [((cc[2] * N + cc[1]) * N + cc[0]) * 12 for cc in c]


def geometry(name):
    """(px, py): per-instruction pixel offsets, shape (64,), and the instruction
    grid (step_x, step_y) over which the 64-pixel pattern tiles the frame"""
    l = np.arange(64)
    if name == '8x8 dense (k_tile)':
        return l % 8, l // 8
    if name == '256x1 stride 4 (lane 4x2, row of lanes)':
        return 4 * l, 0 * l
    if name == '128x1 stride 2 (lane 2x2, row of lanes)':
        return 2 * l, 0 * l
    if name == '32x8 stride 2 (lane 2x2, 16x4 lanes)':
        return 2 * (l % 16), 2 * (l // 16)
    if name == '64x8 stride 4x2 (lane 4x2, 16x4 lanes)':
        return 4 * (l % 16), 2 * (l // 16)
    if name == '16x16 stride 2 (lane 2x2, 8x8 lanes)':
        return 2 * (l % 8), 2 * (l // 8)
    if name == '32x16 stride 4x2 (lane 4x2, 8x8 lanes)':
        return 4 * (l % 8), 2 * (l // 8)
    if name == '64x4 stride 8x1 ... (lane 8x1)':
        return 8 * (l % 8), l // 8
    raise KeyError(name)


GEOMS = ['8x8 dense (k_tile)', '16x16 stride 2 (lane 2x2, 8x8 lanes)', '32x16 stride 4x2 (lane 4x2, 8x8 lanes)',
         '32x8 stride 2 (lane 2x2, 16x4 lanes)', '64x8 stride 4x2 (lane 4x2, 16x4 lanes)',
         '128x1 stride 2 (lane 2x2, row of lanes)', '256x1 stride 4 (lane 4x2, row of lanes)']


def main():
    for kind in sys.argv[1:] or ['smooth', 'real', 'uniform']:
        s = coords(kind)
        offs = corner_offsets(s)
        print(f'== {kind}')
        for g in GEOMS:
            px, py = geometry(g)
            # the pattern has strides; the instruction origins fill the gaps
            stx = int(np.diff(np.unique(px))[0]) if len(np.unique(px)) > 1 else 1
            sty = int(np.diff(np.unique(py))[0]) if len(np.unique(py)) > 1 else 1
            bw, bh = px.max() + stx, py.max() + sty
            xs = [(x0 + a) for x0 in range(0, W - bw + 1, bw) for a in range(stx)]
            ys = [(y0 + b) for y0 in range(0, H - bh + 1, bh) for b in range(sty)]
            xs = np.array(xs)[:, None] + px[None, :]      # (nx, 64)
            ys = np.array(ys)[:, None] + py[None, :]      # (ny, 64)
            tot_lines = 0.0
            cost = 0.0
            ninst = 0
            rng = np.random.default_rng(0)
            sel_y = rng.choice(len(ys), size=min(len(ys), 60), replace=False)
            for yi in sel_y:
                yy = ys[yi]
                for o in offs:
                    v = o[yy[None, :], xs]                  # (nx, 64) byte offsets
                    lo = v // 64
                    hi = (v + 11) // 64
                    both = np.sort(np.concatenate([lo, hi], 1), 1)
                    d = 1 + (np.diff(both, axis=1) != 0).sum(1)
                    tot_lines += d.sum()
                    cost += np.maximum(16.5, 1.07 * d).sum()
                    ninst += len(d)
            print(f'  {g:42s} lines/instr {tot_lines / ninst:6.2f}  est clk/instr {cost / ninst:6.1f}'
                  f'  clk/px (4 gathers) {4 * cost / ninst / 64:5.2f}')


if __name__ == '__main__':
    main()
