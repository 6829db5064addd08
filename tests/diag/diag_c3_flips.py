"""Where the C3 (libplacebo branch, BT.2390) rgba8 download flips come from
(VERDICT r03 item 2), on a 4K smooth frame and the reference's website frame:
the stage-3 value v = 255 x the BT.1886 (target black) encode before the
download's rounding, tile kernel vs oracle, as |dv| in 8-bit code units,
split by how close the oracle's v sits to a rounding boundary and by the
pixel's darkest input PQ code; and the flips themselves (the download code
that differs).  GPU box.  Usage: python tests/diag/diag_c3_flips.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, os.path.join(REPO, 'tests')]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames, frames_from_rgb8  # noqa: E402

LAT = hdr2sdr.generate_lattice(65)
W, H = 3840, 2160
tm = hdr2sdr.Tonemapper(0)
p = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
op = oracle.params_from(p.to_c())
out = {}
for kind in ('smooth', 'website'):
    if kind == 'website':
        z = np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))
        src = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=11)
    tm.set_params(p)
    tm.set_lut(LAT)
    buf = src.to_numpy().buf
    want = np.clip(oracle.debug_float(op, LAT, buf, W, H, 3).astype(np.float64), 0.0, 1.0) * 255.0
    got = tm.debug_float(src.to_torch('cuda'), 3).astype(np.float64) * 255.0
    ok = np.isfinite(want) & np.isfinite(got)
    dv = np.abs(got - want)[ok]
    fw = (want - np.floor(want + 0.5))[ok]                 # oracle's distance from the .5 boundary... (v + 0.5 floored)
    dist = np.abs(np.abs(fw) - 0.5)                        # distance of v + 0.5 to the next integer
    qw = np.floor(want + 0.5)[ok]
    qg = np.floor(got + 0.5)[ok]
    flip = qw != qg
    y = src.to_numpy().y[0].astype(np.int64)
    rec = dict(kind=kind, values=int(ok.sum()),
               dv_pct=[float(np.percentile(dv, q)) for q in (50, 90, 99, 99.9, 99.99, 100)],
               flips=int(flip.sum()), flip_frac=float(flip.mean()),
               flips_within=[int((flip & (dist < e)).sum()) for e in (1e-5, 1e-4, 1e-3, 1e-2)],
               near_ties=[float((dist < e).mean()) for e in (1e-5, 1e-4, 1e-3, 1e-2)])
    # the flips by luma code (dark vs not)
    yy = np.broadcast_to(y[None], want.shape)[ok]
    rec['flip_luma_codes_pct'] = [int(np.percentile(yy[flip], q)) for q in (0, 10, 50, 90, 100)] if flip.any() else []
    rec['dv_by_luma'] = {f'{lo}-{hi}': float(np.percentile(dv[(yy >= lo) & (yy < hi)], 99.9))
                         for lo, hi in ((64, 128), (128, 256), (256, 512), (512, 1024)) if ((yy >= lo) & (yy < hi)).any()}
    print(json.dumps(rec), flush=True)
    out[kind] = rec
os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
with open(os.path.join(REPO, 'gpurun_out', 'diag_c3_flips.json'), 'w') as fh:
    json.dump(out, fh, indent=1)
