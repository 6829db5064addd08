"""Time k_tile variants (libh2s builds with different -D flags) on the C2
workload and diff their outputs against the first variant.

  python scripts/time_variants.py lib_a.so lib_b.so ...
Each variant runs in its own subprocess (H2S_LIB=...)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, time
sys.path.insert(0, os.path.join(REPO, 'hdr-to-sdr_amd')); sys.path.insert(0, REPO)
import numpy as np, torch, hdr2sdr
from hdr2sdr.synth import synth_frames
dev = torch.device('cuda', 0)
tm_name = os.environ.get('TM', 'hable')
p = hdr2sdr.TonemapParams(tonemapper=tm_name, gamma=2.2, bits_in=10, bits_out=10, mode='compat8')
tm = hdr2sdr.Tonemapper(0, p, hdr2sdr.generate_lattice(65))
res = {}
for kind in os.environ.get('KINDS', 'smooth,uniform,edges').split(','):
    if kind == 'website':   # the reference's own 4K HDR frame, 16 copies (as bench.py's real_content line)
        from hdr2sdr.synth import frames_from_rgb8
        z = np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))
        src = frames_from_rgb8(z[z.files[0]], 16, 10, dev)
    else:
        src = synth_frames(kind, 16, 3840, 2160, 10, device=dev, seed=0x5EED)
    dst = hdr2sdr.FrameBatch.empty_torch(16, 3840, 2160, 10, dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(3): tm.process(src, dst, s)
    torch.cuda.synchronize()
    tm.set_timing(True)
    for _ in range(20): tm.process(src, dst, s)
    torch.cuda.synchronize()
    ms = tm.kernel_ms(20); tm.set_timing(False)
    out = dst.buf[[0, 9]].cpu().numpy().astype(np.int32)
    ref = f'/tmp/ref_{tm_name}_{kind}.npy'
    if not os.path.exists(ref):
        np.save(ref, out); d = {'ref': True}
    else:
        r = np.load(ref); diff = np.abs(out - r)
        d = {'max': int(diff.max()), 'ndiff': int((diff > 0).sum()), 'frac': float((diff > 0).mean())}
    res[kind] = {'ms': round(ms, 4), 'mpx': round(16 * 3840 * 2160 / ms / 1e3, 1), **d}
    del src, dst
print('RESULT ' + json.dumps(res))
'''


def main():
    for spec in sys.argv[1:]:
        lib, _, kv = spec.partition('@')   # lib.so[@VAR=val,VAR2=val]
        env = dict(os.environ, H2S_LIB=os.path.abspath(lib))
        for item in filter(None, kv.split(',')):
            k, _, v = item.partition('=')
            env[k] = v
        r = subprocess.run([sys.executable, '-c', 'REPO=%r\n' % REPO + CHILD], env=env, capture_output=True,
                           text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith('RESULT ')]
        if r.returncode != 0 or not line:
            print(os.path.basename(spec), 'FAILED rc', r.returncode, r.stderr[-2000:], flush=True)
            sys.exit(1)
        print(f'{os.path.basename(spec):40s} {line[0][7:]}', flush=True)


if __name__ == '__main__':
    main()
