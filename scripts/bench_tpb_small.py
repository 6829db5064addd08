"""Tiles per block (H2S_OPT_TILES_PER_BLOCK) on the launches whose block count
is a small multiple of the resident slots (256 CUs x 5 blocks): C1 (16 1080p
frames: 2040 blocks at 8 tiles per block = 1.6 block-waves) and C5 (4 8K
frames: 8100 blocks = 6.3 waves).  Kernel ms (HIP events, 20 calls after 3),
two rounds.  GPU box.  Usage: python scripts/bench_tpb_small.py"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

CFGS = {'C1': (dict(tonemapper='reinhard', gamma=1.0, bits_out=8), 1920, 1080, 16, 33, (2, 3, 4, 5, 6, 8, 12)),
        'C5': (dict(tonemapper='hable', gamma=1.0, bits_in=12, bits_out=12, transfer='arib-std-b67'), 7680, 4320, 4, 65,
               (5, 8, 10, 12, 16)),
        'C3_4f': (dict(tonemapper='bt.2390', gamma=1.0, bits_out=10), 3840, 2160, 4, 65, (2, 4, 8, 16))}
res = {}
for rnd in range(2):
    for name, (kw, W, H, nf, n, tpbs) in CFGS.items():
        p = hdr2sdr.TonemapParams(**kw)
        tm = hdr2sdr.Tonemapper(0, p, hdr2sdr.generate_lattice(n))
        src = synth_frames('smooth', nf, W, H, p.bits_in, device='cuda', seed=0x5EED)
        dst = hdr2sdr.FrameBatch.empty_torch(nf, W, H, p.bits_out, 'cuda')
        for tpb in tpbs:
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
        del src, dst
    print(json.dumps(res), flush=True)
