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

# stage dumps at the pixels of the failing chroma blocks (frame 0)
if 'H2S_LIB' not in os.environ:
    n = 177
    lat = hdr2sdr.generate_lattice(n)
    p = hdr2sdr.TonemapParams(tonemapper='mobius')
    src = synth_frames('uniform', 1, W, H, 10, device='cpu', seed=11)
    tm = hdr2sdr.Tonemapper(0, p, lat)
    op = oracle.params_from(p.to_c())
    dst = hdr2sdr.FrameBatch.empty_numpy(1, W, H, 10)
    tm.process(src.to_numpy(), dst)
    got = dst.buf.astype(np.int64).ravel()
    want = oracle.process(op, lat, src.to_numpy().buf, W, H).astype(np.int64).ravel()
    bad = np.flatnonzero(got != want)
    print('1-frame product diffs', bad.size, bad[:20].tolist(), got[bad[:20]].tolist(), want[bad[:20]].tolist())
    g5 = np.asarray(tm.debug_float(src.to_torch("cuda"), 5)).reshape(3, H, W)
    w5 = oracle.debug_float(op, lat, src.to_numpy().buf, W, H, 5).reshape(3, H, W)
    d5 = np.abs(g5 - w5)
    print('stage 5 max diff', float(np.nanmax(d5)), 'count > 0.01', int((d5 > 0.01).sum()))
    o3 = oracle.debug_float(op, lat, src.to_numpy().buf, W, H, 3).reshape(3, H, W)
    for i in bad[:12]:
        if i < W * H:
            y, x = divmod(i, W)
            print(f'  out {i} luma px ({y},{x}) s3 {o3[:, y, x].tolist()} gpu5 {g5[:, y, x].tolist()} ora5 {w5[:, y, x].tolist()}')
            continue
        ci = (i - W * H) % (W * H // 4)
        cy, cx = divmod(ci, W // 2)
        for y in (2 * cy, 2 * cy + 1):
            for x in (2 * cx, 2 * cx + 1):
                print(f'  out {i} px ({y},{x}) s3 {o3[:, y, x].tolist()} gpu5 {g5[:, y, x].tolist()} ora5 {w5[:, y, x].tolist()}')
    tm.close()
