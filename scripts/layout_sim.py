"""Distinct cache lines one tetrahedral lookup touches, per lattice layout
(uniformly random lattice coordinates; DESIGN.md §4.1, uniform content)."""
import numpy as np
rng = np.random.default_rng(1)
N = 65
M = 400000
s = rng.uniform(0, N - 1, size=(M, 3))
i = np.floor(s).astype(np.int64); d = s - i
# tetrahedral corners: c0, c0+e_max, c0+e_max+e_mid, c0+1
order = np.argsort(-d, axis=1)
E = np.eye(3, dtype=np.int64)
c1 = i + E[order[:, 0]]
c2 = c1 + E[order[:, 1]]
c3 = i + 1
corners = [i, c1, c2, c3]
def lin(c, rec): return ((c[:, 2] * N + c[:, 1]) * N + c[:, 0]) * rec
def brick(c, rec, B=(N + 1) // 2, pad=None):
    bsz = pad or rec * 8
    bi = (c[:, 2] >> 1) * B * B + (c[:, 1] >> 1) * B + (c[:, 0] >> 1)
    w = (c[:, 0] & 1) + 2 * (c[:, 1] & 1) + 4 * (c[:, 2] & 1)
    return bi * bsz + w * rec
for name, f, rec in (('linear12', lambda c: lin(c, 12), 12), ('linear16', lambda c: lin(c, 16), 16),
                     ('brick12(96B)', lambda c: brick(c, 12), 12), ('brick16(128B)', lambda c: brick(c, 16), 16),
                     ('brick12 pad128', lambda c: brick(c, 12, pad=128), 12)):
    for line in (64, 128):
        lines = set()
        tot = 0
        offs = [f(c) for c in corners]
        L = np.stack([np.stack([o // line, (o + rec - 1) // line], 1) for o in offs], 1).reshape(M, -1)
        Ls = np.sort(L, axis=1)
        distinct = 1 + (np.diff(Ls, axis=1) != 0).sum(1)
        print(f'{name:16s} line {line:3d}B: distinct lines per pixel {distinct.mean():.3f}')
