"""Build tests/golden/website_frames.npz from the reference's website pair
(`HDR to SDR Website/hdr-frame.png`, `sdr-frame.png`, 3840x2160 RGB8): the
HDR frame as displayed (PQ BT.2020 R'G'B' in 8 bits) and the tool's SDR
output, settings unknown (a plausibility fixture, not a
golden).  Every 8th pixel of both (offset 4), i.e. 480 x 270 samples each.
Also website_hdr_full.npz: the whole HDR frame (3840 x 2160 x 3 uint8), the
real-content input of bench.py's `real_content` line.
Run in the build container, where /root/reference exists:
  python tests/golden/make_website_fixture.py"""
import os

import numpy as np
from PIL import Image

SRC = '/root/reference/HDR to SDR Website'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'website_frames.npz')
OUT_FULL = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'website_hdr_full.npz')


def main():
    arrs = {}
    for key, name in (('hdr', 'hdr-frame.png'), ('sdr', 'sdr-frame.png')):
        im = np.asarray(Image.open(os.path.join(SRC, name)).convert('RGB'))
        arrs[key] = np.ascontiguousarray(im[4::8, 4::8])
        if key == 'hdr':
            np.savez_compressed(OUT_FULL, hdr=np.ascontiguousarray(im))
    np.savez_compressed(OUT, **arrs)
    print(OUT, {k: v.shape for k, v in arrs.items()}, os.path.getsize(OUT), 'bytes')


if __name__ == '__main__':
    main()
