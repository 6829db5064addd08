"""Diagnostic (GPU, not collected by pytest): share of output samples where
the HIP path and the oracle differ, luma and chroma apart, for a few switch
combinations with and without the S6 ordered dither, per content kind."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'hdr-to-sdr_amd'), ROOT, os.path.join(ROOT, 'tests')]
import hdr2sdr  # noqa: E402
from test_gpu_parity import run_both  # noqa: E402

tm = hdr2sdr.Tonemapper(0)
W, H = 128, 64
CASES = [dict(tonemapper='mobius', gamma=1.4, chroma_edge='replicate', bits_out=8),
         dict(tonemapper='mobius', gamma=1.4, bits_out=8),
         dict(tonemapper='hable', gamma=2.2, bits_out=8),
         dict(tonemapper='reinhard', lut_enabled=False, bits_out=8)]
for kw in CASES:
    for dither in ('none', 'ordered'):
        for kind in ('smooth', 'edges', 'ramp', 'uniform'):
            p = hdr2sdr.TonemapParams(**dict(kw, dither=dither))
            got, want, _ = run_both(tm, p, kind, W, H)
            ysz = W * H
            dy = got[:, :ysz] != want[:, :ysz]
            dc = got[:, ysz:] != want[:, ysz:]
            print(f'{str(kw):90s} dither={dither:7s} {kind:7s} luma {dy.mean():.4%} chroma {dc.mean():.4%} '
                  f'all {(got != want).mean():.4%} max {np.abs(got - want).max()}', flush=True)
