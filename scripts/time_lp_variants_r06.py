"""The libplacebo branch's tile kernel on its BASELINE-adjacent configs
(C3 BT.2390 IPT, its max(R,G,B) form, spline, libplacebo hable; 16 4K
frames per call, smooth and uniform content): median ms per call with HIP
events.  The library is whatever H2S_LIB names (lattice-gather build vs the
8-bit table) and H2S_LP_TAB picked the table order (until the linear
order was removed: profiles/r06/ab_patches/lp_tab_linear.patch).  GPU box.
Usage: H2S_LIB=... H2S_LP_TAB=0|1 python scripts/time_lp_variants_r06.py TAG"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

W, H, N = 3840, 2160, 16
lat = hdr2sdr.generate_lattice(65)
CFGS = {'C3': dict(tonemapper='bt.2390'), 'C3_max_rgb': dict(tonemapper='bt.2390', lp_tone='max-rgb'),
        'C3_spline': dict(tonemapper='spline'), 'C2_libplacebo': dict(tonemapper='hable', pipeline='libplacebo')}
res = {'tag': sys.argv[1] if len(sys.argv) > 1 else '?'}
for kind in ('smooth', 'uniform'):
    src = synth_frames(kind, N, W, H, 10, device='cuda', seed=5)
    for name, kw in CFGS.items():
        tm = hdr2sdr.Tonemapper(0, hdr2sdr.TonemapParams(gamma=1.0, bits_out=10, **kw), lat)
        out = tm(src)
        s = torch.cuda.current_stream()
        for _ in range(3):
            tm.process(src, out)
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            tm.process(src, out)
            b.record(s)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        res[f'{name}_{kind}'] = round(ts[len(ts) // 2], 4)
        tm.close()
print(json.dumps(res))
