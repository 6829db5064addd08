"""Checksums of the libplacebo branch's outputs (the configs of
time_lp_variants_r06.py, 4 4K frames of smooth and uniform content and the
website frame) for the library H2S_LIB names: two builds whose lines match
produce identical output.  GPU box.  Usage: H2S_LIB=... python scripts/lp_output_checksum.py TAG"""
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames, frames_from_rgb8  # noqa: E402

W, H, N = 3840, 2160, 4
lat = hdr2sdr.generate_lattice(65)
CFGS = {'C3': dict(tonemapper='bt.2390'), 'C3_max_rgb': dict(tonemapper='bt.2390', lp_tone='max-rgb'),
        'C3_spline': dict(tonemapper='spline'), 'C2_libplacebo': dict(tonemapper='hable', pipeline='libplacebo')}
res = {'tag': sys.argv[1] if len(sys.argv) > 1 else '?'}
for kind in ('smooth', 'uniform', 'website'):
    if kind == 'website':
        src = frames_from_rgb8(np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))['hdr'], N, 10, 'cuda')
    else:
        src = synth_frames(kind, N, W, H, 10, device='cuda', seed=5)
    for name, kw in CFGS.items():
        tm = hdr2sdr.Tonemapper(0, hdr2sdr.TonemapParams(gamma=1.0, bits_out=10, **kw), lat)
        out = tm(src).to_numpy()
        res[f'{name}_{kind}'] = hashlib.sha1(np.ascontiguousarray(out.buf).tobytes()).hexdigest()[:16]
        tm.close()
print(json.dumps(res))
