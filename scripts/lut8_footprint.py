"""Lattice-line footprint of the libplacebo branch's rgba8 codes if lut3d's
8-bit path were one 2^24-entry table (linear r + 256 g + 65536 b, or 4x4x4
bricks): distinct 128-B lines per 8x8 step, per 64x32 tile and per frame,
from the oracle's stage-3 output on C3 (profiles/r03/ablations/lp_lut8_table.log)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'hdr-to-sdr_amd')); sys.path.insert(0, REPO)
import oracle, hdr2sdr
from hdr2sdr.synth import synth_frames, frames_from_rgb8
W, H = 3840, 2160
p = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10)
lat = hdr2sdr.generate_lattice(65)
def codes(kind):
    if kind == 'website':
        rgb = np.load(os.path.join(REPO, 'tests/golden/website_hdr_full.npz'))
        rgb = rgb[rgb.files[0]]
        fb = frames_from_rgb8(rgb, 1, 10)
    else:
        fb = synth_frames(kind, 1, W, H, 10)
    buf = fb.buf.numpy() if hasattr(fb.buf, 'numpy') else np.asarray(fb.buf)
    g = oracle.debug_float(oracle.params_from(p.to_c()), lat, buf, W, H, 3)   # stage 3: encoded R'G'B' before download
    return np.floor(np.clip(g, 0, 1) * 255 + 0.5).astype(np.int64)
def lin(r, g, b): return r + 256 * g + 65536 * b
def brick(r, g, b): return (((b >> 2) << 12 | (g >> 2) << 6 | (r >> 2)) << 6) | (b & 3) << 4 | (g & 3) << 2 | (r & 3)
for kind in ('smooth', 'website', 'uniform'):
    q = codes(kind)
    r, g, b = q[0], q[1], q[2]
    for name, f in (('linear', lin), ('brick', brick)):
        line = (f(r, g, b) * 4) // 128
        # 8x8 steps: distinct lines per step; 64x32 tiles: distinct lines per tile
        st = line[:H // 8 * 8, :].reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        ps = np.mean([len(np.unique(x)) for x in st[::37]])
        tl = line[:H // 32 * 32].reshape(H // 32, 32, W // 64, 64).transpose(0, 2, 1, 3).reshape(-1, 2048)
        pt = np.mean([len(np.unique(x)) for x in tl[::7]])
        tot = len(np.unique(line))
        print(f'{kind:8s} {name:7s} lines/step {ps:6.2f}  lines/tile {pt:7.1f}  distinct lines/frame {tot:8d} ({tot*128/1e6:.1f} MB)')
