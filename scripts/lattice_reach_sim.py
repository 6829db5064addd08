"""How much of the 65^3 lattice one 4K frame of the bench content reaches,
C2 (CPU chain, Hable, gamma 2.2) against C3 (libplacebo branch, BT.2390, IPT;
lut3d's 8-bit coordinates) and C3 on the CPU chain: distinct 128-B lattice
lines per frame, per 64x32 tile, and per 8-tile block run (VERDICT r03 item 6:
where C3's lattice refetch comes from).  Test infrastructure (oracle)."""
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO + '/hdr-to-sdr_amd', REPO, REPO + '/scripts']
os.chdir(REPO)
import oracle, hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames, frames_from_rgb8  # noqa: E402
from geom_sim import corner_offsets  # noqa: E402
N, W, H = 65, 3840, 2160
g = np.linspace(0, 1, N, dtype=np.float32)
LAT = np.stack(np.meshgrid(g, g, g, indexing='ij')[::-1], -1).reshape(-1, 3)
CFG = {'C2': dict(tonemapper='hable', gamma=2.2),
       'C3': dict(tonemapper='bt.2390', bits_out=10),
       'C3_cpu_chain': dict(tonemapper='bt.2390', bits_out=10, pipeline='cpu'),
       'C3_max_rgb': dict(tonemapper='bt.2390', bits_out=10, lp_tone='max-rgb')}
for kind in sys.argv[1:] or ['smooth', 'real']:
    if kind == 'real':
        fb = frames_from_rgb8(np.load('tests/golden/website_hdr_full.npz')['hdr'], 1, 10, 'cpu').to_numpy()
    else:
        fb = synth_frames(kind, 1, W, H, 10, device='cpu', seed=0x5EED).to_numpy()
    for name, kw in CFG.items():
        p = hdr2sdr.TonemapParams(**kw)
        s3 = oracle.debug_float(oracle.params_from(p.to_c()), LAT, fb.buf, W, H, 3).astype(np.float64)
        if p.resolved_pipeline() == 'libplacebo':
            s3 = np.floor(np.clip(np.nan_to_num(s3), 0, 1) * 255 + 0.5) / 255    # the rgba8 download
        s = np.clip(np.nan_to_num(s3) * (N - 1), 0, N - 1 - 1e-4)
        lines = np.stack([o // 128 for o in corner_offsets(s)])          # (4, H, W)
        tiles = lines[:, :H // 32 * 32].reshape(4, H // 32, 32, W // 64, 64).transpose(1, 3, 0, 2, 4).reshape(H // 32, W // 64, -1)
        per_tile = [len(np.unique(tiles[y, x])) for y in range(0, H // 32, 3) for x in range(0, W // 64, 3)]
        run = [len(np.unique(tiles[y, x:x + 8])) for y in range(0, H // 32, 3) for x in range(0, W // 64 - 8, 8)]
        print(f'{kind:6s} {name:13s} frame: {len(np.unique(lines)):6d} lines ({len(np.unique(lines)) * 128 / 2**20:.2f} MB of '
              f'{N**3 * 12 / 2**20:.2f}); per 64x32 tile mean {np.mean(per_tile):.0f}, per 8-tile run {np.mean(run):.0f}', flush=True)
