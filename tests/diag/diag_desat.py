"""Locate GPU-vs-oracle luma samples beyond one pre-eq step for one config
and print the float stages of both at those pixels (GPU box)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import torch  # noqa: E402
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

LAT = hdr2sdr.generate_lattice(65)
W, H = 128, 64
p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=10, desat_luma=sys.argv[1] if len(sys.argv) > 1 else 'bt2020')
src = synth_frames('edges', 2, W, H, 10, device='cpu', seed=11)
tm = hdr2sdr.Tonemapper(0, p, LAT)
dst = hdr2sdr.FrameBatch.empty_torch(2, W, H, 10, 'cuda')
tm.process(src.to_torch('cuda'), dst)
torch.cuda.synchronize()
got = dst.to_numpy().buf.astype(np.int64)
op = oracle.params_from(p.to_c())
want = oracle.process(op, LAT, src.to_numpy().buf, W, H).astype(np.int64)
ysz = W * H
d = np.abs(got[:, :ysz] - want[:, :ysz]) >> 2
idx = np.argwhere(d > 1)
print('luma beyond one 8-bit step:', len(idx))
for f, i in idx[:5]:
    y, x = divmod(int(i), W)
    print(f'frame {f} pixel ({x},{y}) got {got[f, i]} want {want[f, i]}  src Y {src.to_numpy().buf[f, i]}')
    one = hdr2sdr.FrameBatch(np.ascontiguousarray(src.to_numpy().buf[f:f + 1]), W, H, 10)
    print('  codes Y', one.y[0, y, x], 'U', one.u[0, y // 2, x // 2], 'V', one.v[0, y // 2, x // 2])
    for st in (1, 2, 3, 4, 5):
        g = tm.debug_float(one.to_torch('cuda'), st)[:, y, x]
        w = oracle.debug_float(op, LAT, one.buf, W, H, st)[:, y, x]
        print(f'  stage {st}: gpu {g} oracle {w}')
    tm.set_option(1, 0)
    for st in (1, 2, 3):
        g = tm.debug_float(one.to_torch('cuda'), st)[:, y, x]
        print(f'  generic stage {st}: gpu {g}')
    tm.set_option(1, 1)
