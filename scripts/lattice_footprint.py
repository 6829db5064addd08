"""Distinct 128-B lattice lines (12-B Y'CbCr records, 65^3, linear layout) a
tile of W x H pixels touches through its four tetrahedral corners, on the bench
content ('smooth') and the reference's website frame ('real'); 200 random
tiles each.  Compared with the 32 KB L1 of a CU, which holds the five tiles
of its five resident blocks.  Test infrastructure only
(imports the oracle through scripts/geom_sim.py)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
os.chdir(os.path.dirname(HERE))
from geom_sim import coords, corner_offsets  # noqa: E402


def main():
    for kind in sys.argv[1:] or ['smooth', 'real']:
        s = coords(kind)
        offs = corner_offsets(s)
        H, W = s.shape[1:]
        for tw, th in [(64, 32), (128, 32), (128, 64), (256, 64)]:
            rng = np.random.default_rng(0)
            res = []
            for _ in range(200):
                x0 = rng.integers(0, W // tw) * tw
                y0 = rng.integers(0, H // th) * th
                lines = set()
                for o in offs:
                    v = o[y0:y0 + th, x0:x0 + tw].ravel()
                    lines.update((v // 128).tolist())
                    lines.update(((v + 11) // 128).tolist())
                res.append(len(lines))
            res = np.array(res)
            print(f'{kind:6s} tile {tw}x{th}: unique 128-B lines mean {res.mean():.0f} '
                  f'(= {res.mean() * 128 / 1024:.1f} KB), p90 {np.percentile(res, 90):.0f}')


if __name__ == '__main__':
    main()
