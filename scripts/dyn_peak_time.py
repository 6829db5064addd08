import os, sys, time, json
REPO = os.environ.get('GRAFT_REPO_ROOT', '/root/repo')
sys.path.insert(0, os.path.join(REPO, 'hdr-to-sdr_amd')); sys.path.insert(0, REPO)
import torch, hdr2sdr
from hdr2sdr.synth import synth_frames
dev = torch.device('cuda', 0)
res = {}
for tmn in ('bt.2390', 'spline'):
    for pd in (False, True):
        p = hdr2sdr.TonemapParams(tonemapper=tmn, gamma=1.0, bits_out=10, peak_detect=pd, maxcll=4000.0)
        tm = hdr2sdr.Tonemapper(0, p, hdr2sdr.generate_lattice(65))
        src = synth_frames('smooth', 16, 3840, 2160, 10, device=dev, seed=0x5EED)
        dst = hdr2sdr.FrameBatch.empty_torch(16, 3840, 2160, 10, dev)
        s = torch.cuda.current_stream(dev)
        for _ in range(3): tm.process(src, dst, s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10): tm.process(src, dst, s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        res[f'{tmn}{"_dyn" if pd else ""}'] = {'ms_per_16': round(ms, 3), 'mpx_s': round(16 * 3840 * 2160 / ms / 1e3, 1)}
        tm.close()
print(json.dumps(res))
