"""The dynamic-peak statistics kernel alone, for a kernel trace of a library
variant (H2S_LIB, scripts/build_ablation.sh): h2s_peak_stats over 16 4K
frames of the bench content (or argv[1]: a synth kind, or website; argv[2]: blocks per frame), REPS times with the percentile histogram and
REPS times without (pd_percentile 100).  GPU box.
Usage: H2S_LIB=... rocprofv3 --kernel-trace ... -- python3 scripts/bench_peak_kernel.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

W, H, N, REPS = 3840, 2160, 16, 40
lat = hdr2sdr.generate_lattice(65)
KIND = sys.argv[1] if len(sys.argv) > 1 else 'smooth'
if KIND == 'website':   # the reference's own HDR frame (tests/golden), repeated per frame
    import numpy as np
    from hdr2sdr.synth import frames_from_rgb8
    src = frames_from_rgb8(np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))['hdr'], N, 10, 'cuda')
else:
    src = synth_frames(KIND, N, W, H, 10, device='cuda', seed=5)
for pct in (float('nan'), 100.0):
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10, peak_detect=True, maxcll=4000.0,
                              pd_percentile=pct)
    tm = hdr2sdr.Tonemapper(0, p, lat)
    if len(sys.argv) > 2:   # partial records (blocks) per frame
        from hdr2sdr import _abi
        tm.set_option(_abi.OPT_TEST_PEAK_BLOCKS, int(sys.argv[2]))
    for _ in range(REPS):
        tm.peak_stats(src)
    torch.cuda.synchronize()
    tm.close()
print('lib', os.environ.get('H2S_LIB', 'product'), 'done')
