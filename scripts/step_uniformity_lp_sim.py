"""Share of the libplacebo branch's 8x8 steps (C3, BT.2390) whose rgba8 codes
put all 64 pixels in one lattice cell and tetrahedron, from the oracle's
stage-3 output (profiles/r03/ablations/step_uniformity.txt)."""
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO + '/hdr-to-sdr_amd', REPO]
import oracle, hdr2sdr
from hdr2sdr.synth import synth_frames, frames_from_rgb8
W,H=3840,2160
p=hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10)
lat=hdr2sdr.generate_lattice(65)
for kind in ('smooth','website'):
    if kind=='website':
        z=np.load(REPO+'/tests/golden/website_hdr_full.npz'); fb=frames_from_rgb8(z[z.files[0]],1,10)
    else: fb=synth_frames(kind,1,W,H,10)
    g=oracle.debug_float(oracle.params_from(p.to_c()), lat, fb.buf.numpy(), W, H, 3)
    q=np.floor(np.clip(g,0,1)*255+0.5)
    s=np.minimum(q*(1/255)*64,64).astype(np.float32)
    c=np.minimum(np.floor(s),63).astype(np.int64); d=s-c
    cell=c[0]+65*c[1]+65*65*c[2]
    tet=(d[0]>d[1]).astype(int)*4+(d[1]>d[2]).astype(int)*2+(d[0]>d[2]).astype(int)
    key=cell*8+tet
    st=key[:H//8*8].reshape(H//8,8,W//8,8).transpose(0,2,1,3).reshape(-1,64)
    print(kind, 'LP steps uniform cell+tet %.3f' % (st==st[:,:1]).all(1).mean())
