"""Diagnostic (GPU, not collected by pytest): the CPU chain with the LUT off
on 'edges' content, with and without the S6 ordered dither — where the HIP
path and the oracle disagree on chroma, with both sides' stage-4 floats."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'hdr-to-sdr_amd'), ROOT, os.path.join(ROOT, 'tests')]
import torch  # noqa: E402
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

W, H = 128, 64
tm = hdr2sdr.Tonemapper(0)
for dither in ('none', 'ordered'):
    for tmo in ('reinhard', 'hable'):
        p = hdr2sdr.TonemapParams(tonemapper=tmo, lut_enabled=False, bits_out=8, dither=dither)
        src_cpu = synth_frames('edges', 2, W, H, 10, device='cpu', seed=11)
        tm.set_params(p)
        dst = hdr2sdr.FrameBatch.empty_torch(2, W, H, 8, 'cuda')
        tm.process(src_cpu.to_torch('cuda'), dst)
        torch.cuda.synchronize()
        got = dst.to_numpy().buf.astype(np.int64)
        want = oracle.process(oracle.params_from(p.to_c()), None, src_cpu.to_numpy().buf, W, H).astype(np.int64)
        ysz = W * H
        dy = np.abs(got[:, :ysz] - want[:, :ysz])
        dc = np.abs(got[:, ysz:] - want[:, ysz:])
        print(f'dither={dither} tm={tmo}: luma >1: {(dy > 1).sum()}  chroma >1: {(dc > 1).sum()}  '
              f'chroma max {dc.max()}', flush=True)
        idx = np.argwhere(dc[0] > 1)[:4]
        for (i,) in idx:
            plane = i // (ysz // 4)
            j = i % (ysz // 4)
            cy, cx = divmod(j, W // 2)
            print(f'  plane {plane + 1} ({cx},{cy}): got {got[0, ysz + i]} want {want[0, ysz + i]}', flush=True)
            src = src_cpu.to_numpy()
            print('   Y codes', src.y[0, 2 * cy:2 * cy + 2, 2 * cx:2 * cx + 2].tolist(), 'U', int(src.u[0, cy, cx]),
                  'V', int(src.v[0, cy, cx]), flush=True)
            for st in (2, 4):
                o = oracle.debug_float(oracle.params_from(p.to_c()), None, src.buf, W, H, st)
                g = tm.debug_float(src_cpu.to_torch('cuda'), st) if hasattr(tm, 'debug_float') else None
                print(f'   stage {st} oracle', o[:, 2 * cy:2 * cy + 2, 2 * cx:2 * cx + 2].reshape(3, 4).tolist(), flush=True)
                if g is not None:
                    g = np.asarray(g.cpu() if hasattr(g, 'cpu') else g)
                    print(f'   stage {st} hip   ', g[:, 2 * cy:2 * cy + 2, 2 * cx:2 * cx + 2].reshape(3, 4).tolist(),
                          flush=True)
