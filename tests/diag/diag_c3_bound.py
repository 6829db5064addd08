"""Can a per-value bound predict where the tile kernel's C3 download may
round the other way?  (a near-tie path needs a window
that holds every flip and little else.)

The tile kernel's stage-3 value v (255 x the BT.1886 encode against the
target black, before the rgba8 rounding) differs from the oracle's by |dv|.
Model: the IPT form's LMS relative error d propagates to the linear channel
r_c through the LMS -> RGB row, |dr_c| <= d S_c, S_c = sum_k |l2r[c, k]|
LMS_k; then through the encode, |dv| <= (v + 255 b) / (2.4 r_c) |dr_c|.
So |dv| <= d B_c with B_c = (v + 255 b) S_c / (2.4 r_c); d_eff = |dv| / B_c
should be bounded.  Reports d_eff's percentiles, and for a window of d B_c
with d at several values: the share of values it flags and of the flips it
catches.  Cheaper proxies are tried too: S_c <= |l2r row| lmax.
GPU box.  Usage: python tests/diag/diag_c3_bound.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, os.path.join(REPO, 'tests')]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames, frames_from_rgb8  # noqa: E402
from ipt_cond import ipt_matrices  # noqa: E402

LAT = hdr2sdr.generate_lattice(65)
W, H = 3840, 2160
tm = hdr2sdr.Tonemapper(0)
p = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
op = oracle.params_from(p.to_c())
tm.set_params(p)
tm.set_lut(LAT)
r2l, l2r = ipt_matrices()
tw, tb = 203.0, 0.203
lb = (tb / tw) ** (1 / 2.4)
b = lb / (1 - lb)
out = {}
for kind in ('smooth', 'website'):
    if kind == 'website':
        z = np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))
        src = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=11)
    buf = src.to_numpy().buf
    w2 = oracle.debug_float(op, LAT, buf, W, H, 2).astype(np.float64)
    w3 = np.clip(oracle.debug_float(op, LAT, buf, W, H, 3).astype(np.float64), 0, 1) * 255
    g3 = np.clip(tm.debug_float(src.to_torch('cuda'), 3).astype(np.float64), 0, 1) * 255
    lms = np.einsum('kc,chw->khw', r2l, w2)
    S = np.einsum('ck,khw->chw', np.abs(l2r), np.abs(lms))
    lmax = np.abs(lms).max(axis=0, keepdims=True)
    S2 = np.abs(l2r).sum(1)[:, None, None] * lmax
    r = np.abs(w2)
    dv = np.abs(g3 - w3)
    ok = np.isfinite(dv) & (r > 0)
    flip = np.floor(g3 + 0.5) != np.floor(w3 + 0.5)
    dist = np.abs((w3 + 0.5) - np.round(w3 + 0.5))
    rec = {'kind': kind, 'flips': int(flip[ok].sum())}
    for name, Sx in (('S', S), ('L1_lmax', S2)):
        with np.errstate(divide='ignore', invalid='ignore'):
            B = (w3 + 255 * b) * Sx / (2.4 * r)
            deff = dv / B
        d = deff[ok & (dv > 0)]
        rec[f'{name}_deff_pcts_50_99_999_max'] = [float(np.percentile(d, q)) for q in (50, 99, 99.9, 100)]
        for dd in (3e-5, 1e-4, 3e-4):
            win = dd * B
            flag = ok & (dist < win)
            rec[f'{name}_d{dd:g}'] = {'flag_share': float(flag[ok].mean()),
                                      'flips_caught': float((flag & flip)[ok].sum() / max(1, (flip & ok).sum())),
                                      'pixels_flagged': float(flag.any(axis=0).mean())}
    print(json.dumps(rec), flush=True)
    out[kind] = rec
tm.close()
with open(os.path.join(REPO, 'gpurun_out', 'diag_c3_bound.json'), 'w') as fh:
    json.dump(out, fh, indent=1)
