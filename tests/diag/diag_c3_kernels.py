"""C3 (libplacebo branch, BT.2390, 4K) output parity of both kernels against
the oracle: the tile kernel (k_tile<..., LP = 1>) and the generic kernel
(H2S_OPT_FAST_PATH = 0: the IPT form in double, ocml powf), on a smooth
synthetic frame and the reference's website frame.  Per kernel: output
samples beyond one 10-bit step, max diff, and the stage-3 (pre-download)
disagreement |dv| in 8-bit codes with the download flips it causes.
GPU box.  Usage: python tests/diag/diag_c3_kernels.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, os.path.join(REPO, 'tests')]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames, frames_from_rgb8  # noqa: E402

LAT = hdr2sdr.generate_lattice(65)
W, H = 3840, 2160
tm = hdr2sdr.Tonemapper(0)
p = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
op = oracle.params_from(p.to_c())
tm.set_params(p)
tm.set_lut(LAT)
res = {}
for kind in ('smooth', 'website'):
    if kind == 'website':
        z = np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))
        src = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=11)
    buf = src.to_numpy().buf
    want = oracle.process(op, LAT, buf, W, H).astype(np.int64)
    w3 = np.clip(oracle.debug_float(op, LAT, buf, W, H, 3).astype(np.float64), 0.0, 1.0) * 255.0
    dsrc = src.to_torch('cuda')
    for fast in (1, 0):
        tm.set_option(_abi.OPT_FAST_PATH, fast)
        got = tm(dsrc).to_numpy().buf.astype(np.int64)
        g3 = np.clip(tm.debug_float(dsrc, 3).astype(np.float64), 0.0, 1.0) * 255.0
        d = np.abs(got - want)
        dv = np.abs(g3 - w3)
        ok = np.isfinite(dv)
        flips = int((np.floor(g3 + 0.5) != np.floor(w3 + 0.5))[ok].sum())
        rec = dict(kind=kind, kernel='k_tile' if fast else 'k_process', beyond_1_step=int((d > 1).sum()),
                   max_diff=int(d.max()), exact=float((d == 0).mean()), download_flips=flips,
                   dv_p50_p99_p999_max=[float(np.percentile(dv[ok], q)) for q in (50, 99, 99.9, 100)])
        print(json.dumps(rec), flush=True)
        res[f'{kind}_{rec["kernel"]}'] = rec
tm.set_option(_abi.OPT_FAST_PATH, 1)
tm.close()
os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
with open(os.path.join(REPO, 'gpurun_out', 'diag_c3_kernels.json'), 'w') as fh:
    json.dump(res, fh, indent=1)
