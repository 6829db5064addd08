"""C3 (4K BT.2390, libplacebo branch, 16 frames) under H2S_OPT_LP_EXACT 0
(tile kernel), 1 (tile kernel's near-tie instances + the exact pass over the
listed quads) and 2 (generic kernel): ms per 16 frames on the smooth bench
content and on the reference's website frame (HIP events around the call),
and each mode's output against the oracle on one frame of each content
(samples beyond one output step, max diff).  GPU box.
Usage: python scripts/bench_lp_exact.py [--windows 3000,6000,12000]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
import oracle  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import frames_from_rgb8, synth_frames  # noqa: E402


def timed(tm, src, dst, reps=10):
    s = torch.cuda.current_stream()
    for _ in range(2):
        tm.process(src, dst)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        tm.process(src, dst)
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--windows', default='6000')
    args = ap.parse_args()
    W, H = 3840, 2160
    lat = hdr2sdr.generate_lattice(65)
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10)
    op = oracle.params_from(p.to_c())
    z = np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))
    one = {'smooth': synth_frames('smooth', 1, W, H, 10, device='cpu', seed=11),
           'website': frames_from_rgb8(z[z.files[0]], 1, 10)}
    want = {k: oracle.process(op, lat, f.to_numpy().buf, W, H).astype(np.int64) for k, f in one.items()}
    batch = {'smooth': synth_frames('smooth', 16, W, H, 10, device='cuda', seed=0x5EED),
             'website': frames_from_rgb8(z[z.files[0]], 16, 10, 'cuda')}
    tm = hdr2sdr.Tonemapper(0, p, lat)
    res = {}
    runs = [(0, None), (2, None)] + [(1, int(w)) for w in args.windows.split(',')]
    for mode, win in runs:
        tm.set_option(_abi.OPT_LP_EXACT, mode)
        if win:
            tm.set_option(_abi.OPT_TEST_NT_WINDOW, win)
        tag = f'mode{mode}' + (f'_w{win}' if win else '')
        rec = {}
        for kind in ('smooth', 'website'):
            dst = tm(batch[kind])
            rec[f'{kind}_ms'] = round(timed(tm, batch[kind], dst), 4)
            got = tm(one[kind].to_torch('cuda')).to_numpy().buf.astype(np.int64)
            d = np.abs(got - want[kind])
            rec[f'{kind}_beyond_1'] = int((d > 1).sum())
            rec[f'{kind}_max_diff'] = int(d.max())
        res[tag] = rec
        print(json.dumps({tag: rec}), flush=True)
    tm.close()
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(REPO, 'gpurun_out', 'bench_lp_exact.json'), 'w') as fh:
        json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
