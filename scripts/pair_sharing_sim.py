"""Share of neighbouring pixel pairs / 2x2 quads whose tetrahedral lookups use
the same lattice cell and tetrahedron (the same four records), per content:
the upper bound on the gather traffic that a lane owning two pixels could
skip by reusing its first pixel's records.  Test
infrastructure only (imports the oracle through scripts/geom_sim.py)."""
import sys, numpy as np, os
HERE = os.path.dirname(os.path.abspath(__file__)); sys.path.insert(0, HERE); os.chdir(os.path.dirname(HERE))
from geom_sim import coords
for kind in ['smooth','real','uniform']:
    s = coords(kind)
    i = np.floor(s).astype(np.int64); d = s - i
    order = np.argsort(-d, axis=0)
    key = ((i[2]*65 + i[1])*65 + i[0])*8 + order[0]*3 + order[1]   # cell + tetrahedron (max, mid axes)
    cell = (i[2]*65 + i[1])*65 + i[0]
    h = (key[:, 0::2] == key[:, 1::2]).mean()
    v = (key[0::2, :] == key[1::2, :]).mean()
    hc = (cell[:, 0::2] == cell[:, 1::2]).mean()
    q = ((key[0::2,0::2]==key[0::2,1::2]) & (key[0::2,0::2]==key[1::2,0::2]) & (key[0::2,0::2]==key[1::2,1::2])).mean()
    print(f'{kind:8s} horizontal pair same cell+tetra {h:.3f} (same cell {hc:.3f}), vertical {v:.3f}, whole 2x2 quad {q:.3f}')
