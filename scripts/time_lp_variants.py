"""Time libplacebo-branch (C3) k_tile variants (libh2s builds with different
-D flags, scripts/build_variants.sh) and count their output disagreements
with the oracle: per variant, ms per 16 4K frames (smooth; the tile kernel's
HIP-event time), and on one smooth frame and the reference's website frame
the samples beyond one output step and the max diff.  Each variant runs in its
own subprocess (H2S_LIB=...).  GPU box.
Usage: python scripts/time_lp_variants.py lib_a.so lib_b.so ..."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json
REPO = os.environ['REPO']
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import numpy as np, torch, hdr2sdr, oracle
from hdr2sdr.synth import synth_frames, frames_from_rgb8
dev = torch.device('cuda', 0)
lat = hdr2sdr.generate_lattice(65)
p = hdr2sdr.TonemapParams(tonemapper=os.environ.get('TM', 'bt.2390'), gamma=1.0, bits_out=10)
tm = hdr2sdr.Tonemapper(0, p, lat)
res = {}
src = synth_frames('smooth', 16, 3840, 2160, 10, device=dev, seed=0x5EED)
dst = hdr2sdr.FrameBatch.empty_torch(16, 3840, 2160, 10, dev)
s = torch.cuda.current_stream(dev)
for _ in range(3): tm.process(src, dst, s)
torch.cuda.synchronize(); tm.set_timing(True)
for _ in range(20): tm.process(src, dst, s)
torch.cuda.synchronize(); res['ms'] = round(tm.kernel_ms(20), 4); tm.set_timing(False)
op = oracle.params_from(p.to_c())
for kind in ('smooth', 'website'):
    if kind == 'website':
        z = np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))
        f = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        f = synth_frames('smooth', 1, 3840, 2160, 10, device='cpu', seed=11)
    want = oracle.process(op, lat, f.to_numpy().buf, 3840, 2160).astype(np.int64)
    got = tm(f.to_torch('cuda')).to_numpy().buf.astype(np.int64)
    d = np.abs(got - want)
    res[kind] = {'beyond_1_step': int((d > 1).sum()), 'max_diff': int(d.max()), 'differ': int((d > 0).sum())}
tm.close()
print(json.dumps(res))
'''


def main():
    out = {}
    for lib in sys.argv[1:]:
        env = dict(os.environ, H2S_LIB=os.path.abspath(lib), REPO=REPO)
        r = subprocess.run([sys.executable, '-c', CHILD], env=env, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stdout, r.stderr[-3000:], flush=True)
            raise SystemExit(f'{lib}: rc {r.returncode}')
        out[os.path.basename(lib)] = json.loads(r.stdout.strip().splitlines()[-1])
        print(json.dumps({os.path.basename(lib): out[os.path.basename(lib)]}), flush=True)


if __name__ == '__main__':
    main()
