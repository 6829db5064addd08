"""LDS-box variant of scripts/box_fit_sim.py: a 4x4x4-node box anchored at
lane 0's cell (cells -1..+1 per axis, 768 B of LDS per wave, the only size that
keeps 5 blocks per CU), and min-anchored boxes, against the scalar-record
steps.  Test infrastructure (oracle)."""
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
    g = oracle.debug_float(oracle.params_from(p.to_c()), lat, fb.buf.numpy() if hasattr(fb.buf,'numpy') else fb.buf, W, H, 3)
    s = np.clip(np.nan_to_num(g), 0, 1) * 64
    c = np.minimum(np.floor(s), 63).astype(np.int64); d = s - c
    tet = (d[0] > d[1]).astype(int) * 4 + (d[1] > d[2]).astype(int) * 2 + (d[0] > d[2]).astype(int)
    def steps(a):
        return a[:H // 8 * 8].reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    cr, cg, cb, tt = steps(c[0]), steps(c[1]), steps(c[2]), steps(tet)
    key = (cr * 65 + cg) * 65 + cb
    uni = ((key == key[:, :1]) & (tt == tt[:, :1])).all(1)
    for lo, hi in [(-1, 1), (0, 2), (-2, 1)]:
        fit = np.ones(len(cr), bool)
        for a in (cr, cg, cb):
            dd = a - a[:, :1]
            fit &= ((dd >= lo) & (dd <= hi)).all(1)
        print(kind, f'anchor lane0 cells [{lo},{hi}]: fits {fit.mean():.3f}, fits & not uniform {(fit & ~uni).mean():.3f}, uniform {uni.mean():.3f}')
    # min-anchored 3 cells per axis
    fit = np.ones(len(cr), bool)
    for a in (cr, cg, cb):
        fit &= (a.max(1) - a.min(1)) <= 2
    print(kind, f'min-anchored 3 cells/axis: fits & not uniform {(fit & ~uni).mean():.3f}')
    fit = np.ones(len(cr), bool)
    for a in (cr, cg, cb):
        fit &= (a.max(1) - a.min(1)) <= 1
    print(kind, f'min-anchored 2 cells/axis (27 nodes): fits & not uniform {(fit & ~uni).mean():.3f}')
