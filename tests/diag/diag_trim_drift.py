"""Does the round-4 VALU-trim build move C2's output towards or away from the
oracle?  Two 4K smooth frames (the full-size C2 check's input), each library
variant (H2S_LIB list in argv) in a child process, diffed against the oracle
and against the first variant.  GPU box.  Usage:
python tests/diag/diag_trim_drift.py lib1.so lib2.so"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
CHILD = r'''
import sys, numpy as np
sys.path[:0] = [REPO + '/hdr-to-sdr_amd', REPO]
import hdr2sdr
from hdr2sdr.synth import synth_frames
p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=10)
src = synth_frames('smooth', 2, 3840, 2160, 10, device='cpu', seed=0x5EED).to_numpy()
tm = hdr2sdr.Tonemapper(0, p, hdr2sdr.generate_lattice(65))
dst = hdr2sdr.FrameBatch.empty_numpy(2, 3840, 2160, 10)
tm.process(src, dst)
np.save(OUT, dst.buf)
'''


def main():
    import oracle
    import hdr2sdr
    from hdr2sdr.synth import synth_frames
    p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=10)
    src = synth_frames('smooth', 2, 3840, 2160, 10, device='cpu', seed=0x5EED).to_numpy()
    want = oracle.process(oracle.params_from(p.to_c()), hdr2sdr.generate_lattice(65), src.buf, 3840, 2160).astype(np.int64)
    first = None
    for lib in sys.argv[1:]:
        out = f'/tmp/trim_drift_{os.path.basename(lib)}.npy'
        env = dict(os.environ, H2S_LIB=os.path.abspath(lib))
        code = CHILD.replace('REPO', repr(REPO)).replace('OUT', repr(out))
        subprocess.run([sys.executable, '-c', code], env=env, check=True, timeout=300)
        got = np.load(out).astype(np.int64)
        rec = dict(lib=os.path.basename(lib), vs_oracle_ndiff=int((got != want).sum()),
                   vs_oracle_maxabs=int(np.abs(got - want).max()))
        if first is None:
            first = got
        else:
            d = got != first
            rec.update(vs_first_ndiff=int(d.sum()), closer=int((d & (got == want)).sum()),
                       further=int((d & (first == want)).sum()))
        print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
