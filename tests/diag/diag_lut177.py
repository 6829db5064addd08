"""Isolate the N = 177 tile-kernel failure (round-4 VALU trims): Mobius,
uniform content, 64x32, 177^3 lattice, GPU vs oracle; reports the output
samples that are not multiples of the 8->10-bit shift.  Run per library
variant (H2S_LIB=...).  GPU box."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, os.path.join(REPO, 'tests')]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

W, H = 64, 32
for n in (129, 177):
    lat = hdr2sdr.generate_lattice(n)
    p = hdr2sdr.TonemapParams(tonemapper='mobius')
    src = synth_frames('uniform', 2, W, H, 10, device='cpu', seed=11).to_numpy()
    tm = hdr2sdr.Tonemapper(0, p, lat)
    dst = hdr2sdr.FrameBatch.empty_numpy(2, W, H, 10)
    tm.process(src, dst)
    tm.close()
    got = dst.buf.astype(np.int64)
    want = oracle.process(oracle.params_from(p.to_c()), lat, src.buf, W, H).astype(np.int64)
    bad = np.flatnonzero(got % 4)
    d = np.abs(got - want)
    print(f'N={n}: lib={os.path.basename(os.environ.get("H2S_LIB", "in-tree"))} max diff {d.max()} '
          f'ndiff {(d > 0).sum()} non-mult-4 {bad.size} at {bad[:8].tolist()} got {got.flat[bad[:8]].tolist()} '
          f'want {want.flat[bad[:8]].tolist()}', flush=True)
