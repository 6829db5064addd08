"""How the libplacebo branch's tone curve is applied to colour, tried on the
reference's website pair (tests/golden/website_frames.npz; see
tests/test_website_fixture.py).  Diagnostic, CPU only, float64 numpy: the
BT.2390 curve comes from the oracle (libplacebo defaults, fitted peak), and is
applied as
  max   gain f(max RGB)/max RGB on R, G, B (the restatement in libh2s/oracle),
  luma  gain f(Y)/Y with BT.2020 luminance,
  chan  f per channel,
  ipt   f on the intensity of IPT-PQ (HPE LMS, Ebner-Fairchild matrix), P/T
        scaled by the intensity ratio,
then BT.1886 against the target black, 8-bit download, lut3d's 8-bit
tetrahedral path.  --screenshot selects the screenshot model of the test.
Usage: python tests/diag/website_models.py [--screenshot bt601] max luma chan ipt"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402

M1, M2 = 2610 / 16384, 2523 / 4096 * 128
C1, C2, C3 = 3424 / 4096, 2413 / 4096 * 32, 2392 / 4096 * 32
KRB = {'601': (0.299, 0.114), '709': (0.2126, 0.0722), '2020': (0.2627, 0.0593)}
M2020_709 = np.array([[1.6604910021, -0.5876411388, -0.0728498633], [-0.1245504745, 1.1328998971, -0.0083494226],
                      [-0.0181507634, -0.1005788980, 1.1187296614]])


def eotf(e):
    e = np.clip(np.nan_to_num(e), 0, 1)
    xp = e ** (1 / M2)
    return (np.maximum(xp - C1, 0) / (C2 - C3 * xp)) ** (1 / M1)


def oetf(y):
    ym = np.clip(y, 0, None) ** M1
    return ((C1 + C2 * ym) / (1 + C3 * ym)) ** M2


def rgb2yuv(m):
    kr, kb = KRB[m]
    kg = 1 - kr - kb
    return np.array([[kr, kg, kb], [-kr / (2 * (1 - kb)), -kg / (2 * (1 - kb)), 0.5],
                     [0.5, -kg / (2 * (1 - kr)), -kb / (2 * (1 - kr))]])


def reinterpret(a, b):
    """R'G'B' a decoder made with matrix a -> the R'G'B' matrix b gives."""
    return np.linalg.inv(rgb2yuv(b)) @ rgb2yuv(a)


def tetra(lat, n, s):
    """vf_lut3d interp_tetrahedral, vectorised (red fastest)."""
    s = np.clip(np.nan_to_num(s), 0, n - 1)
    i = np.minimum(np.floor(s).astype(int), n - 2)
    f = s - i
    r, g, b = i[..., 0], i[..., 1], i[..., 2]
    x, y, z = f[..., 0:1], f[..., 1:2], f[..., 2:3]

    def c(dr, dg, db):
        return lat[(r + dr) + n * (g + dg) + n * n * (b + db)]
    c000, c111 = c(0, 0, 0), c(1, 1, 1)
    X, Y, Z = x[..., 0], y[..., 0], z[..., 0]
    case = np.select([(X > Y) & (Y > Z), (X > Y) & (X > Z), X > Y, Z > Y, Z > X], [0, 1, 2, 3, 4], 5)
    forms = [lambda: (1 - x) * c000 + (x - y) * c(1, 0, 0) + (y - z) * c(1, 1, 0) + z * c111,
             lambda: (1 - x) * c000 + (x - z) * c(1, 0, 0) + (z - y) * c(1, 0, 1) + y * c111,
             lambda: (1 - z) * c000 + (z - x) * c(0, 0, 1) + (x - y) * c(1, 0, 1) + y * c111,
             lambda: (1 - z) * c000 + (z - y) * c(0, 0, 1) + (y - x) * c(0, 1, 1) + x * c111,
             lambda: (1 - y) * c000 + (y - z) * c(0, 1, 0) + (z - x) * c(0, 1, 1) + x * c111,
             lambda: (1 - y) * c000 + (y - x) * c(0, 1, 0) + (x - z) * c(1, 1, 0) + z * c111]
    out = np.zeros(s.shape)
    for k, fn in enumerate(forms):
        m = case == k
        if m.any():
            out[m] = fn()[m]
    return out


def run(E, lat, model, peak, tw=203.0):
    op = oracle.params_from(hdr2sdr.TonemapParams(tonemapper='bt.2390', peak=peak).to_c())
    sig = np.geomspace(1e-7, 100.0, 4000)
    cur = np.array([oracle.tone_curve(op, float(v)) for v in sig])   # npl units -> target-white units

    def f(v):
        return np.interp(np.log(np.maximum(v, 1e-7)), np.log(sig), cur)
    L = eotf(E) * 100.0
    if model == 'max':
        s = np.maximum(L.max(-1), 1e-6)
        T = L * (f(s) / s)[..., None]
    elif model == 'luma':
        y = np.maximum(L @ np.array([0.2627, 0.6780, 0.0593]), 1e-6)
        T = L * (f(y) / y)[..., None]
    elif model == 'chan':
        T = f(L)
    else:
        m2x = np.array([[0.636958, 0.144617, 0.168881], [0.262700, 0.677998, 0.059302], [0, 0.028073, 1.060985]])
        hpe = np.array([[0.4002, 0.7076, -0.0808], [-0.2263, 1.1653, 0.0457], [0, 0, 0.9182]])
        r2l = hpe @ m2x
        l2i = np.array([[0.4, 0.4, 0.2], [4.455, -4.851, 0.396], [0.8056, 0.3572, -1.1628]])
        ipt = oetf(L / 100.0 @ r2l.T) @ l2i.T
        i0 = ipt[..., 0].copy()
        i1 = oetf(f(eotf(i0) * 100.0) * tw / 10000)
        ipt[..., 0] = i1
        ipt[..., 1:] *= np.where(i0 > 1e-6, i1 / np.maximum(i0, 1e-6), 1.0)[..., None]
        T = (eotf(ipt @ np.linalg.inv(l2i).T) @ np.linalg.inv(r2l).T) * 10000 / tw
    lb = (1 / 1000) ** (1 / 2.4)
    a, b = (1 - lb) ** 2.4, lb / (1 - lb)
    q = np.floor(np.clip((np.maximum(T, 0) / a) ** (1 / 2.4) - b, 0, 1) * 255 + 0.5)
    n = round(lat.shape[0] ** (1 / 3))
    return np.clip(np.trunc(tetra(lat, n, q / 255 * (n - 1)) * 255), 0, 255)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--screenshot', default='bt2020', choices=['bt2020', 'bt601'])
    ap.add_argument('models', nargs='*', default=['max', 'luma', 'chan', 'ipt'])
    a = ap.parse_args()
    d = np.load(os.path.join(REPO, 'tests', 'golden', 'website_frames.npz'))
    E, S = d['hdr'].astype(np.float64) / 255.0, d['sdr'].astype(np.float64)
    hm, sm = ('2020', '709') if a.screenshot == 'bt2020' else ('601', '601')
    E = np.clip(E @ reinterpret(hm, '2020').T, 0, 1)
    lat = hdr2sdr.generate_lattice(65).reshape(-1, 3).astype(np.float64)
    for model in a.models:
        fits = []
        for pk in (4.0, 5.0, 6.0, 8.0, 10.0, 13.0):
            o = np.clip(np.round(run(E, lat, model, pk) @ reinterpret('709', sm).T), 0, 255)
            fits.append((float(np.abs(o - S).mean()), pk, (o - S).reshape(-1, 3).mean(0)))
        m, pk, bias = min(fits, key=lambda t: t[0])
        print(f'{a.screenshot:7s} {model:5s} best MAE {m:.3f}/255 at peak {pk:g} (x100 nits), bias {np.round(bias, 2)}')


if __name__ == '__main__':
    with np.errstate(invalid='ignore'):
        main()
