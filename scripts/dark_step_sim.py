"""Share of k_tile's 8x8 steps holding a channel in the PQ table's first
segment (0 < E' < 1/128: linear below ~0.0015 nits), where the cubic table
cannot hold 1e-3 relative: the cost driver of any
ballot-gated dark path.  From the oracle's stage-1 linear values on the bench's
smooth content, uniform noise and the reference's website frame."""
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO + '/hdr-to-sdr_amd', REPO]
import oracle, hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames, frames_from_rgb8  # noqa: E402
W, H = 3840, 2160
p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
op = oracle.params_from(p.to_c())
LAT = hdr2sdr.generate_lattice(65)
thr = oracle.pq_eotf(1.0 / 128) * 1e4 / 100.0     # units of npl = 100 nits
print('first-segment bound (units of npl): %.4g' % thr)
for kind in ('smooth', 'uniform', 'website'):
    if kind == 'website':
        z = np.load(REPO + '/tests/golden/website_hdr_full.npz')
        fb = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        fb = synth_frames(kind, 1, W, H, 10, device='cpu', seed=0x5EED)
    buf = fb.buf.numpy() if hasattr(fb.buf, 'numpy') else fb.buf
    lin = oracle.debug_float(op, LAT, buf, W, H, 1)
    dark = ((lin > 0) & (lin < thr)).any(axis=0)
    st = dark[:H // 8 * 8].reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    tiles = dark[:H // 32 * 32].reshape(H // 32, 32, W // 64, 64).any(axis=(1, 3))
    print(f'{kind}: pixels with a dark channel {dark.mean():.4f}, 8x8 steps holding one {st.any(1).mean():.4f}, '
          f'64x32 tiles holding one {tiles.mean():.4f}')
