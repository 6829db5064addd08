"""Worst stage-N relative error of k_tile's debug instance vs the oracle for
one config (GPU box): prints that pixel's codes and stages 1-3 on both."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

LAT = hdr2sdr.generate_lattice(65)
W, H = 128, 64
kind, stage = sys.argv[1], int(sys.argv[2])
import json
p = hdr2sdr.TonemapParams(**(json.loads(sys.argv[3]) if len(sys.argv) > 3 else dict(tonemapper='hable', gamma=2.2,
                                                                                      bits_out=10)))
src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=3)
tm = hdr2sdr.Tonemapper(0, p, LAT)
op = oracle.params_from(p.to_c())
g = tm.debug_float(src.to_torch('cuda'), stage).astype(np.float64)
w = oracle.debug_float(op, LAT, src.to_numpy().buf, W, H, stage).astype(np.float64)
lin = oracle.debug_float(op, LAT, src.to_numpy().buf, W, H, 1).astype(np.float64)
wts = {'rgb': (1, 1, 1), 'bt2020': (0.2627, 0.6780, 0.0593), 'bt709': (0.2126, 0.7152, 0.0722)}[p.desat_luma]
with np.errstate(invalid='ignore', divide='ignore'):
    luma = wts[0] * lin[0] + wts[1] * lin[1] + wts[2] * lin[2]
    kappa = np.nan_to_num(np.where(luma > p.desat, luma / (luma - p.desat), 0.0), nan=0.0, posinf=0.0)
    skip = (np.abs(luma - p.desat) < 0.02 * luma) | ~(np.nanmax(np.abs(np.nan_to_num(lin, nan=np.inf)), axis=0) < 1e6)
    gain = np.maximum(1.0, np.nan_to_num(np.nanmax(np.abs(w), axis=0) / np.nanmax(np.abs(lin), axis=0), nan=1.0, posinf=1.0))
    rel = np.abs(g - w) / ((1e-3 + 4e-5 * kappa) * np.abs(w) + 2e-7 * gain)      # the float test's tolerance ratio
    rel[:, skip] = 0
print('kappa max among kept', kappa[~skip].max())
rel = np.nan_to_num(rel, nan=0.0, posinf=0.0)
c, y, x = np.unravel_index(int(np.argmax(rel)), rel.shape)
print('worst', rel[c, y, x], 'channel', c, 'pixel', (x, y))
print('codes Y', src.to_numpy().y[0, y, x], 'U', src.to_numpy().u[0, y // 2, x // 2], 'V', src.to_numpy().v[0, y // 2, x // 2])
for st in (1, 2, 3):
    gs = tm.debug_float(src.to_torch('cuda'), st)[:, y, x]
    ws = oracle.debug_float(op, LAT, src.to_numpy().buf, W, H, st)[:, y, x]
    print(f'stage {st}: gpu {gs} oracle {ws}')
tm.set_option(1, 0)
print('generic stage 1:', tm.debug_float(src.to_torch('cuda'), 1)[:, y, x])
print('generic stage 2:', tm.debug_float(src.to_torch('cuda'), 2)[:, y, x])
