"""A/B of the peak-statistics kernel forms (H2S_OPT_TEST_PEAK_FORM) and the
dynamic-peak overhead of C3 (16 4K frames per call): per form, the time of
h2s_process with peak_detect against the static call, HIP events on the call's
stream, median of runs.  Run under rocprofv3 --kernel-trace for per-kernel
durations.  GPU box.  Usage: python scripts/bench_peak_stats.py"""
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
lat = hdr2sdr.generate_lattice(65)
src = synth_frames('smooth', N, W, H, 10, device='cuda', seed=5)
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


for dyn in (False, True):
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10, peak_detect=dyn, maxcll=4000.0)
    tm = hdr2sdr.Tonemapper(0, p, lat)
    out = tm(src)            # allocates a device batch of the right shape
    forms = (0, 1, 2) if dyn else (0,)   # 0: quad units (default), 1: round-5 row chunks, 2: quad, 4 in flight
    for form in forms:
        tm.set_option(_abi.OPT_TEST_PEAK_FORM, form)
        res[f'{"dyn" if dyn else "static"}_form{form}_ms'] = round(timed(tm, out), 4)
        print(json.dumps(res), flush=True)
    if dyn:   # partial records (blocks) per frame, quad form
        tm.set_option(_abi.OPT_TEST_PEAK_FORM, 0)
        for nb in (128, 256, 64):
            tm.set_option(_abi.OPT_TEST_PEAK_BLOCKS, nb)
            res[f'dyn_form0_blocks{nb}_ms'] = round(timed(tm, out), 4)
            print(json.dumps(res), flush=True)
    tm.close()
# the statistics alone (h2s_peak_stats: the finish kernel without IIR / curve
# records), and without the histogram (pd_percentile 100), for the trace
for pct in (float('nan'), 100.0):
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10, peak_detect=True, maxcll=4000.0,
                              pd_percentile=pct)
    tm = hdr2sdr.Tonemapper(0, p, lat)
    for _ in range(20):
        tm.peak_stats(src)
    tm.close()
res['dyn_minus_static_form0'] = round(res['dyn_form0_ms'] - res['static_form0_ms'], 4)
res['dyn_minus_static_form1'] = round(res['dyn_form1_ms'] - res['static_form0_ms'], 4)  # round 5's row form
print(json.dumps(res))
