"""Share of k_tile's 8x8 steps whose 64 pixels' lattice cells fit one
wave-box of <= 64 lattice nodes (box-LDS steps), against the cell+tet-uniform
(scalar-record) steps, from the oracle's stage-3 coordinates of C2 on the
bench's smooth content, uniform noise and the reference's website frame."""
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO + '/hdr-to-sdr_amd', REPO]
import oracle, hdr2sdr
from hdr2sdr.synth import synth_frames, frames_from_rgb8


def pow2ceil(x):
    return 1 << int(np.ceil(np.log2(max(x, 1))))


W, H = 3840, 2160
p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
lat = hdr2sdr.generate_lattice(65)
kinds = sys.argv[1:] or ['smooth', 'website', 'uniform']
for kind in kinds:
    if kind == 'website':
        z = np.load(REPO + '/tests/golden/website_hdr_full.npz')
        fb = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        fb = synth_frames(kind, 1, W, H, 10)
    g = oracle.debug_float(oracle.params_from(p.to_c()), lat, fb.buf.numpy(), W, H, 3)
    s = np.clip(np.nan_to_num(g), 0, 1) * 64
    c = np.minimum(np.floor(s), 63).astype(np.int64)
    d = s - c
    tet = (d[0] > d[1]).astype(int) * 4 + (d[1] > d[2]).astype(int) * 2 + (d[0] > d[2]).astype(int)
    def steps(a):
        return a[:H // 8 * 8].reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    cr, cg, cb, tt = steps(c[0]), steps(c[1]), steps(c[2]), steps(tet)
    key = (cr * 65 + cg) * 65 + cb
    uni = ((key == key[:, :1]) & (tt == tt[:, :1])).all(1)
    n = [a.max(1) - a.min(1) + 2 for a in (cr, cg, cb)]
    exact = n[0] * n[1] * n[2] <= 64
    pr = np.array([pow2ceil(x) for x in n[0]]); pg = np.array([pow2ceil(x) for x in n[1]])
    p2 = pr * pg * n[2] <= 64
    p2b = pr * pg * n[2] <= 128
    print(f'{kind}: steps {len(uni)}  uniform(cell+tet) {uni.mean():.3f}  box<=64 nodes exact {exact.mean():.3f}'
          f'  pow2(r,g)*nb<=64 {p2.mean():.3f}  (not uniform & fits {(p2 & ~uni).mean():.3f})  <=128 {p2b.mean():.3f}'
          f'  mean extents {n[0].mean():.2f} {n[1].mean():.2f} {n[2].mean():.2f}')
