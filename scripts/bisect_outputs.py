"""Which commit moved the C2 output between rounds 2 and 3 (VERDICT r03 item
3: checksum 19488649569692 -> 19488649575748).  Each staged package under
scripts/bisect/<commit>/hdr2sdr (that commit's Python host + its libh2s.so,
built from its own sources) converts the same two 4K smooth frames with the C2
params; the outputs are diffed against the first commit's and the oracle's.
Usage (GPU box): python scripts/bisect_outputs.py c1 c2 ..."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, os, numpy as np
sys.path.insert(0, PKG)
import hdr2sdr
buf = np.load(SRC)
W, H = 3840, 2160
p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_in=10, bits_out=10)
tm = hdr2sdr.Tonemapper(0, p, hdr2sdr.generate_lattice(65))
src = hdr2sdr.FrameBatch(buf, W, H, 10)
dst = hdr2sdr.FrameBatch.empty_numpy(buf.shape[0], W, H, 10)
tm.process(src, dst)
np.save(OUT, dst.buf)
'''


def main():
    sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
    from hdr2sdr.synth import synth_frames
    import oracle
    import hdr2sdr
    out_dir = os.path.join(REPO, 'gpurun_out', 'bisect')
    os.makedirs(out_dir, exist_ok=True)
    src = os.path.join('/tmp', 'bisect_src.npy')
    buf = synth_frames('smooth', 2, 3840, 2160, 10, device='cpu', seed=0x5EED).to_numpy().buf
    np.save(src, np.ascontiguousarray(buf))
    p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_in=10, bits_out=10)
    want = oracle.process(oracle.params_from(p.to_c()), hdr2sdr.generate_lattice(65), buf, 3840, 2160).astype(np.int64)
    outs = {}
    for c in sys.argv[1:]:
        pkg = os.path.join(REPO, 'scripts', 'bisect', c) if c != 'HEAD' else os.path.join(REPO, 'hdr-to-sdr_amd')
        out = f'/tmp/bisect_{c}.npy'
        code = f'PKG={pkg!r}; SRC={src!r}; OUT={out!r}\n' + CHILD
        r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(c, 'FAILED', r.stderr[-1500:], flush=True)
            continue
        outs[c] = np.load(out).astype(np.int64)
    first = next(iter(outs))
    rows = []
    for c, o in outs.items():
        d0 = o - outs[first]
        dw = o - want
        rec = dict(commit=c, vs_first_ndiff=int((d0 != 0).sum()), vs_oracle_ndiff=int((dw != 0).sum()),
                   vs_oracle_frac=float((dw != 0).mean()), sum=int(o.sum()))
        if c != first:
            prev = list(outs)[list(outs).index(c) - 1]
            dp = o - outs[prev]
            idx = np.flatnonzero(dp)
            rec['vs_prev'] = prev
            rec['vs_prev_ndiff'] = int(idx.size)
            ysz = 3840 * 2160
            fsz = ysz * 3 // 2
            rec['vs_prev_luma'] = int(((idx % fsz) < ysz).sum())
            rec['vs_prev_maxabs'] = int(np.abs(dp).max(initial=0))
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    with open(os.path.join(out_dir, 'bisect.jsonl'), 'w') as fh:
        for r in rows:
            fh.write(json.dumps(r) + '\n')


if __name__ == '__main__':
    main()
