"""Stage-2 disagreement of the IPT tone form (lp_tone ipt) between the GPU
kernels and the oracle: in units of its float32 conditioning (the LMS -> RGB
row's absolute sum times the pixel's LMS), and the pixels the float test's
tolerance rejects (GPU box).  Usage: python tests/diag/diag_ipt.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO, os.path.join(REPO, 'tests')]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402
from ipt_cond import ipt_channel_scale  # noqa: E402

EPS_IPT = 2e-5
LAT = hdr2sdr.generate_lattice(65)
W, H = 128, 64
tm = hdr2sdr.Tonemapper(0)
for cfg in (dict(tonemapper='bt.2390', bits_out=10), dict(tonemapper='spline', bits_in=12, bits_out=12,
                                                          transfer='arib-std-b67')):
    p = hdr2sdr.TonemapParams(**cfg)
    op = oracle.params_from(p.to_c())
    for kind in ('uniform', 'edges', 'ramp', 'smooth'):
        src = synth_frames(kind, 1, W, H, p.bits_in, device='cpu', seed=3)
        tm.set_params(p)
        tm.set_lut(LAT)
        want = oracle.debug_float(op, LAT, src.to_numpy().buf, W, H, 2).astype(np.float64)
        lin = oracle.debug_float(op, LAT, src.to_numpy().buf, W, H, 1).astype(np.float64)
        scale = ipt_channel_scale(want)
        with np.errstate(invalid='ignore', divide='ignore'):
            gain = np.maximum(1.0, np.nan_to_num(np.nanmax(np.abs(want), axis=0) / np.nanmax(np.abs(lin), axis=0),
                                                 nan=1.0, posinf=1.0))
        tol = 1e-3 * np.abs(want) + 2e-7 * gain[None] + EPS_IPT * scale
        for fast in (1, 0):
            tm.set_option(_abi.OPT_FAST_PATH, fast)
            got = tm.debug_float(src.to_torch('cuda'), 2).astype(np.float64)
            err = np.abs(got - want)
            ok = np.isfinite(want) & np.isfinite(got) & (np.nanmax(np.abs(np.nan_to_num(lin, nan=np.inf)), axis=0) < 1e6)[None]
            r = np.where(ok, (err - 1e-3 * np.abs(want)) / np.maximum(scale, 1e-30), 0)
            name = 'k_tile' if fast else 'k_debug'
            print(cfg['tonemapper'], kind, name,
                  'err/cond p50 %.2e p99 %.2e max %.2e' % tuple(np.percentile(r[ok], [50, 99, 100])), flush=True)
            bad = ok & (err > tol)
            for c, y, x in list(zip(*np.nonzero(bad)))[:3]:
                codes = (src.to_numpy().y[0, y, x], src.to_numpy().u[0, y // 2, x // 2], src.to_numpy().v[0, y // 2, x // 2])
                print(f'   reject ch{c} ({x},{y}) codes {codes} lin {lin[:, y, x]} want {want[:, y, x]} '
                      f'got {got[:, y, x]} tol {tol[c, y, x]:.3g} scale {scale[c, y, x]:.3g} gain {gain[y, x]:.3g}')
tm.set_option(_abi.OPT_FAST_PATH, 1)
tm.close()
