"""C3 (4K BT.2390 on the libplacebo branch, 65^3 LUT, 16 device frames per
call): the tile kernel (default) against the exact path (H2S_OPT_LP_EXACT:
the generic kernel, stages 1-3 in double), HIP events on the call's stream,
median of runs.  GPU box.  Usage: python scripts/time_lp_exact.py"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

W, H, N = 3840, 2160, 16
src = synth_frames('smooth', N, W, H, 10, device='cuda', seed=5)
p = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10)
tm = hdr2sdr.Tonemapper(0, p, hdr2sdr.generate_lattice(65))
out = tm(src)
res = {}
for name, exact, reps in (('tile', 0, 30), ('lp_exact', 1, 5)):
    tm.set_option(_abi.OPT_LP_EXACT, exact)
    s = torch.cuda.current_stream()
    tm.process(src, out)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        tm.process(src, out)
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    res[f'{name}_ms_per_16_frames'] = round(ts[len(ts) // 2], 4)
res['ratio'] = round(res['lp_exact_ms_per_16_frames'] / res['tile_ms_per_16_frames'], 2)
print(json.dumps(res))
