"""A/B of H2S_OPT_TILES_PER_BLOCK (64 x 32 tiles one k_tile block walks) per
configuration: kernel ms per 16 4K frames (HIP events, 20 calls after 3),
rounds alternating.  GPU box.  Usage: python scripts/bench_tpb.py"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

CFGS = {'C2': dict(tonemapper='hable', gamma=2.2, bits_out=10),
        'C3': dict(tonemapper='bt.2390', gamma=1.0, bits_out=10),
        'C3_spline': dict(tonemapper='spline', gamma=1.0, bits_out=10)}
src = synth_frames('smooth', 16, 3840, 2160, 10, device='cuda', seed=0x5EED)
dst = hdr2sdr.FrameBatch.empty_torch(16, 3840, 2160, 10, 'cuda')
lat = hdr2sdr.generate_lattice(65)
res = {}
for rnd in range(2):
    for name, kw in CFGS.items():
        tm = hdr2sdr.Tonemapper(0, hdr2sdr.TonemapParams(**kw), lat)
        for tpb in (4, 8, 16):
            tm.set_option(_abi.OPT_TILES_PER_BLOCK, tpb)
            for _ in range(3):
                tm.process(src, dst)
            torch.cuda.synchronize()
            tm.set_timing(True)
            for _ in range(20):
                tm.process(src, dst)
            torch.cuda.synchronize()
            res.setdefault(f'{name}_tpb{tpb}', []).append(round(tm.kernel_ms(20), 4))
            tm.set_timing(False)
        tm.close()
    print(json.dumps(res), flush=True)
