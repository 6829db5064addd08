"""k_tile time per 16 / 64 4K frames (C2) against tiles per block, for the
libh2s named by H2S_LIB (e.g. the copy-only build of scripts/build_variants.sh)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import torch  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr import _abi  # noqa: E402
from hdr2sdr.synth import synth_frames  # noqa: E402

dev = torch.device('cuda', 0)
tm = hdr2sdr.Tonemapper(0, hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2), hdr2sdr.generate_lattice(65))
for nf in (16, 64):
    src = synth_frames('smooth', nf, 3840, 2160, 10, device=dev, seed=1)
    dst = hdr2sdr.FrameBatch.empty_torch(nf, 3840, 2160, 10, dev)
    for tpb in (1, 2, 4, 8, 16, 32):
        tm.set_option(_abi.OPT_TILES_PER_BLOCK, tpb)
        s = torch.cuda.current_stream(dev)
        for _ in range(3):
            tm.process(src, dst, s)
        torch.cuda.synchronize()
        tm.set_timing(True)
        for _ in range(10):
            tm.process(src, dst, s)
        torch.cuda.synchronize()
        ms = tm.kernel_ms(10)
        tm.set_timing(False)
        print(f'{os.path.basename(os.environ.get("H2S_LIB", "libh2s.so"))} frames {nf} tpb {tpb}: {ms:.4f} ms '
              f'{nf * 3840 * 2160 * 6 / ms / 1e9:.2f} TB/s', flush=True)
    del src, dst
tm.close()
