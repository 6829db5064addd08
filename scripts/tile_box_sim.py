"""The per-tile lattice-cell cache in LDS that VERDICT r03 item 4 describes:
for each 64x32 tile, the bounding box of its pixels' lattice cells (from the
oracle's stage-3 coordinates, i.e. the *exact* box -- a box derived in the
kernel from the tile's code ranges can only be larger), how often it fits an
LDS budget, and how many 8x8 steps it would take off the gather path that the
scalar-record steps do not already (C2, bench smooth content and the website
frame).  Test infrastructure (oracle)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO + '/hdr-to-sdr_amd', REPO]
import oracle, hdr2sdr
from hdr2sdr.synth import synth_frames, frames_from_rgb8
W, H = 3840, 2160
p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
lat = hdr2sdr.generate_lattice(65)
for kind in ['smooth', 'website']:
    if kind == 'website':
        z = np.load(REPO + '/tests/golden/website_hdr_full.npz'); fb = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        fb = synth_frames(kind, 1, W, H, 10, device='cpu', seed=0x5EED)
    buf = fb.buf.numpy() if hasattr(fb.buf,'numpy') else fb.buf
    g = oracle.debug_float(oracle.params_from(p.to_c()), lat, buf, W, H, 3)
    s = np.clip(np.nan_to_num(g), 0, 1) * 64
    c = np.minimum(np.floor(s), 63).astype(np.int64)
    T = c[:, :H//32*32].reshape(3, H//32, 32, W//64, 64)
    lo = T.min(axis=(2, 4)); hi = T.max(axis=(2, 4))
    nodes = np.prod(hi - lo + 2, axis=0)
    for budget in (216, 420, 640, 1024):
        print(kind, f'tiles whose true cell box fits {budget} nodes ({budget*12/1024:.1f} KB): {(nodes <= budget).mean():.3f}')
    print(kind, 'median box nodes', np.median(nodes), 'p25', np.percentile(nodes, 25))
    d = s - c
    tet = (d[0] > d[1]).astype(int) * 4 + (d[1] > d[2]).astype(int) * 2 + (d[0] > d[2]).astype(int)
    key = (c[0] * 65 + c[1]) * 65 + c[2]
    def steps(a):
        return a[:H // 8 * 8].reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(H // 8, W // 8, 64)
    ks, ts = steps(key), steps(tet)
    uni = ((ks == ks[..., :1]) & (ts == ts[..., :1])).all(-1)          # (H/8, W/8)
    uni_t = uni[:H//32*4].reshape(H//32, 4, W//64, 8)                   # tile = 4 x 8 steps
    nonuni_per_tile = (~uni_t).sum(axis=(1, 3))
    for budget in (420, 1024):
        fit = nodes <= budget
        print(kind, f'budget {budget}: share of all steps that are non-uniform AND in a fitting tile: {(nonuni_per_tile * fit).sum() / uni.size:.3f} (non-uniform steps overall {(~uni).mean():.3f})')
