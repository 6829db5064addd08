"""How much of a C3 frame a near-tie repair of the tile kernel would re-run
("re-try the ballot-gated near-tie repair with the
window set by the tile kernel's own bound"): the share of pixels with some
rgba8 download channel whose exact value (oracle.lp_download) lies within
the k_tile bound (float_gate.lp_stage3_bound, the bound tests/lp_gate.py
attributes with) of a rounding boundary, and the share of 8x8 steps (one
wave's 64 lanes) holding at least one such pixel -- the steps a ballot-gated
exact re-run would take.  CPU (oracle only).
Usage: python tests/diag/diag_near_tie_window.py > profiles/r06/near_tie_window.txt"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, os.path.join(REPO, 'tests')]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from float_gate import Planes, lattice, lp_stage3_bound  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

W, H = 1024, 512
print(f'C3 (bt.2390, libplacebo branch, IPT form), {W}x{H}, k_tile bound')
print('| content | pixels with a channel within the bound of a tie | 8x8 steps with such a pixel | '
      'bound median / p99 (8-bit codes) |')
print('|---|---|---|---|')
for kind in ('smooth', 'uniform', 'ramp'):
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10, pipeline='libplacebo')
    op = oracle.params_from(p.to_c())
    src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=5).to_numpy().buf
    P = Planes(p, src, W, H, 65)
    xq = oracle.lp_download(op, lattice(65), src, W, H)
    ys, xs = np.mgrid[0:H, 0:W]
    ys, xs = ys.ravel(), xs.ravel()
    b = lp_stage3_bound(p, 'k_tile', P, ys, xs) * 255.0
    x = xq[:, ys, xs]
    near = (np.abs(x - np.round(x)) <= b).any(axis=0)
    steps = near.reshape(H // 8, 8, W // 8, 8).any(axis=(1, 3)).mean()
    print(f'| {kind} | {near.mean():.2%} | {steps:.1%} | {np.median(b):.4f} / {np.percentile(b, 99):.3f} |')
