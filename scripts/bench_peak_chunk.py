"""A/B of the dynamic-peak schedule on C3 (16 4K frames per call, BT.2390 on
the libplacebo branch): H2S_OPT_TEST_PEAK_CHUNK (frames per pipelined chunk,
0 = whole batch) and H2S_OPT_TEST_PEAK_BLOCKS (statistics blocks per frame).
Per setting the median time of h2s_process with peak_detect against the
static call (HIP events on the call's stream), and whether output and peak
state are bit-identical to the first setting's (3 calls from a reset state,
content with a scene cut).  GPU box.
Usage: python scripts/bench_peak_chunk.py [chunk[:blocks] ...]"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

W, H, N, REPS = 3840, 2160, 16, 30
SETS = [tuple(int(v) for v in (a.split(':') + ['64'])[:2]) for a in sys.argv[1:]] or [(0, 64), (1, 64), (2, 64), (4, 64), (8, 64)]
lat = hdr2sdr.generate_lattice(65)
src = synth_frames('smooth', N, W, H, 10, device='cuda', seed=5)
# a scene cut: frames 8.. from other content, darker
alt = synth_frames('uniform', N, W, H, 10, device='cuda', seed=9)
cut = synth_frames('smooth', N, W, H, 10, device='cuda', seed=5)
half = cut.buf.shape[0] // 2
cut.buf[half:] = alt.buf[half:] // 2
res = {}


def timed(tm, dst):
    s = torch.cuda.current_stream()
    for _ in range(3):
        tm.process(src, dst)
    ts = []
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        tm.process(src, dst)
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def sequence(tm, dst):
    tm.reset_peak()
    outs = []
    for batch in (src, cut, src):
        tm.process(batch, dst)
        torch.cuda.synchronize()
        outs.append(dst.buf.clone())
    return outs, tm.peak_state()


for dyn in (False, True):
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10, peak_detect=dyn, maxcll=4000.0)
    tm = hdr2sdr.Tonemapper(0, p, lat)
    out = tm(src)
    if not dyn:
        res['static_ms'] = round(timed(tm, out), 4)
        print(json.dumps(res), flush=True)
        tm.close()
        continue
    ref = None
    for ch, nb in SETS:
        tm.set_option(_abi.OPT_TEST_PEAK_CHUNK, ch)
        tm.set_option(_abi.OPT_TEST_PEAK_BLOCKS, nb)
        outs, state = sequence(tm, out)
        if ref is None:
            ref = (outs, state)
        key = f'dyn_chunk{ch}_blocks{nb}'
        res[key + '_ms'] = round(timed(tm, out), 4)
        res[key + '_identical'] = bool(all(torch.equal(a, b) for a, b in zip(outs, ref[0])) and state == ref[1])
        res[key + '_state_peak_rel'] = abs(state['peak'] - ref[1]['peak']) / ref[1]['peak']
        res[key + '_minus_static'] = round(res[key + '_ms'] - res['static_ms'], 4)
        print(json.dumps(res), flush=True)
    tm.close()
print(json.dumps(res))
