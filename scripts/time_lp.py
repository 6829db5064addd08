import sys, os
sys.path[:0]=['/root/repo/hdr-to-sdr_amd','/root/repo']
REPO=os.environ.get('GRAFT_REPO_ROOT','/root/repo'); sys.path[:0]=[os.path.join(REPO,'hdr-to-sdr_amd'),REPO]
import torch, hdr2sdr
from hdr2sdr.synth import synth_frames
from hdr2sdr import _abi
dev=torch.device('cuda',0)
tm=hdr2sdr.Tonemapper(0)
src=synth_frames('smooth',16,3840,2160,10,device=dev,seed=1)
dst=hdr2sdr.FrameBatch.empty_torch(16,3840,2160,10,dev)
for name,kw,fast in (('C3 ipt tile',dict(tonemapper='bt.2390'),1),('C3 ipt generic',dict(tonemapper='bt.2390'),0),
                     ('C3 max generic',dict(tonemapper='bt.2390',lp_tone='max-rgb'),0),
                     ('C3 ipt lut off',dict(tonemapper='bt.2390',lut_enabled=False),1),('C3 max lut off',dict(tonemapper='bt.2390',lut_enabled=False,lp_tone='max-rgb'),1)):
    tm.set_params(hdr2sdr.TonemapParams(**kw)); tm.set_lut(hdr2sdr.generate_lattice(65))
    tm.set_option(_abi.OPT_FAST_PATH,fast)
    s=torch.cuda.current_stream(dev)
    for _ in range(2): tm.process(src,dst,s)
    torch.cuda.synchronize(); tm.set_timing(True)
    for _ in range(5): tm.process(src,dst,s)
    torch.cuda.synchronize(); print(name, round(tm.kernel_ms(5),3),'ms', flush=True); tm.set_timing(False)
tm.set_option(_abi.OPT_FAST_PATH,1)
