"""The generic kernel's residual C3 disagreements with the oracle (4K smooth
frame): for every output sample more than one step off, the pixel's input
codes and stage 1 / 2 / 3 values on both sides (float32 bit patterns), so
that the first stage that differs is visible.  GPU box.
Usage: python tests/diag/diag_c3_generic_flips.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, os.path.join(REPO, 'tests')]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

LAT = hdr2sdr.generate_lattice(65)
W, H = 3840, 2160
tm = hdr2sdr.Tonemapper(0)
p = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
op = oracle.params_from(p.to_c())
tm.set_params(p)
tm.set_lut(LAT)
tm.set_option(_abi.OPT_FAST_PATH, 0)
src = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=11)
buf = src.to_numpy().buf
dsrc = src.to_torch('cuda')
want = oracle.process(op, LAT, buf, W, H).astype(np.int64)
got = tm(dsrc).to_numpy().buf.astype(np.int64)
d = np.abs(got - want)[0]
ysz = W * H
bad = np.flatnonzero(d > 1)
pix = set()
for i in bad:
    if i < ysz:
        pix.add((i // W, i % W))
    else:
        j = (i - ysz) % (ysz // 4)
        cy, cx = j // (W // 2), j % (W // 2)
        pix.add((2 * cy, 2 * cx))
planes = {s: (oracle.debug_float(op, LAT, buf, W, H, s), tm.debug_float(dsrc, s)) for s in (1, 2, 3)}
fr = src.to_numpy()
out = []
for (y, x) in sorted(pix)[:40]:
    rec = {'y': int(y), 'x': int(x), 'codes': [int(fr.y[0, y, x]), int(fr.u[0, y // 2, x // 2]), int(fr.v[0, y // 2, x // 2])]}
    for s, (o, g) in planes.items():
        ov, gv = o[:, y, x].astype(np.float32), g[:, y, x].astype(np.float32)
        rec[f's{s}'] = {'oracle': [float(v) for v in ov], 'gpu': [float(v) for v in gv],
                        'ulps': [int(a) - int(b) for a, b in zip(ov.view(np.int32), gv.view(np.int32))]}
    out.append(rec)
    print(json.dumps(rec), flush=True)
print(json.dumps({'beyond_1_step': int(len(bad)), 'pixels': len(pix)}))
tm.close()
