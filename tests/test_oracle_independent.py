"""A second, independent restatement of the CPU chain, in float64 numpy,
checked against the C oracle (oracle/h2s_oracle.c) on whole small frames.

Test infrastructure only, like the oracle.  It is written from the stage
definitions of SURVEY.md §8(a) T1-T10, not from the C code's structure:
  * S1 (zscale t=linear:npl=100, src/utils.py:39): limited-range BT.2020-NCL
    Y'CbCr, chroma bilinear (left-sited horizontally, centre-sited
    vertically, zimg edge rule), ST 2084 EOTF x 10000/npl, or HLG inverse OETF +
    OOTF (gamma 1.2, BT.2100 luma) x 1000/npl;
  * S2 (tonemap=, vf_tonemap): desat 2 on the r+g+b luma, sig = max(R,G,B),
    Reinhard / Hable / Mobius with their defaults, peak 10;
  * S3 (zscale t=bt709): max(x, 0)^(1/2.4);
  * S4 (lut3d interp=tetrahedral, src/utils.py:40): the tetrahedron of the
    sorted fractions (a formulation without the six-way case split);
  * S6 (swscale to yuv420p): BT.709 limited range, 2x2 chroma mean, round;
  * S7 (eq=gamma, src/utils.py:41): vf_eq's 256-entry table;
  * S8 (-pix_fmt, src/ffmpeg_command.py:355-360): the 8-bit code shifted.
Also the native quantiser, the LUT off (legacy closed form, its matrix
derived here from the primaries) and the weighted desat luma.  Measured: the
two agree exactly on 14 of the 27 frames here, and the others differ in at
most 5 of 6144 samples per plane, by one step (float32 vs float64 rounding); nearest-neighbour chroma, a one-pixel siting shift or peak 9
instead of 10 each change 270-5000 samples of the same frame.  The
libplacebo branch (C3's structure with BT.2390 as the max(R,G,B) gain or on
the IPT-PQ intensity, matrices derived here from the primaries and HPE rows:
BT.1886 encode against the target black, rgba8 download, lut3d's truncating
8-bit path, Y'CbCr at the output depth) agrees to <= 10 of 6144 samples per
plane, within the lattice's step for an rgba8 code rounded the other way;
knee offset 0.5 or a 100-nit white instead changes 1000-4600 samples.  Contents
with super-white codes (the 'edges' kind) are left out: there the C
oracle follows vf_tonemap's float32 overflow (inf/NaN then lut3d's
sanitising), which a float64 statement does not reproduce.  Two restatements
in different precisions and formulations agreeing this closely is what this pins: it catches
indexing, siting and stage-order errors in the C oracle, which the GPU
parity tests would otherwise inherit.  It does not pin either against
ffmpeg (parity unpinned)."""
import numpy as np
import pytest

import hdr2sdr
import oracle
from hdr2sdr.synth import synth_frames

TM = {'reinhard': 4, 'hable': 5, 'mobius': 6}
LAT = {}


def lattice(n):
    if n not in LAT:
        LAT[n] = hdr2sdr.generate_lattice(n).astype(np.float64).reshape(n, n, n, 3)  # [b][g][r]
    return LAT[n]


def upsample(c):
    """4:2:0 plane (ch, cw) -> (2ch, 2cw): horizontal left-sited bilinear,
    vertical centre-sited (1/4, 3/4); index -1 mirrors to 1, n clamps to n-1."""
    ch, cw = c.shape
    k = np.arange(cw)
    nxt = np.minimum(k + 1, cw - 1)
    h = np.empty((ch, 2 * cw))
    h[:, 0::2] = c
    h[:, 1::2] = 0.5 * c + 0.5 * c[:, nxt]
    m = np.arange(ch)
    up = np.abs(m - 1)                      # -1 -> 1
    dn = np.minimum(m + 1, ch - 1)
    v = np.empty((2 * ch, 2 * cw))
    v[0::2] = 0.25 * h[up] + 0.75 * h
    v[1::2] = 0.75 * h + 0.25 * h[dn]
    return v


def pq_eotf(e):
    m1, m2, c1, c2, c3 = 2610 / 16384, 2523 / 4096 * 128, 3424 / 4096, 2413 / 4096 * 32, 2392 / 4096 * 32
    xp = np.power(np.maximum(e, 0.0), 1.0 / m2)
    y = np.power(np.maximum(xp - c1, 0.0) / np.maximum(c2 - c3 * xp, np.finfo(np.float32).tiny), 1.0 / m1)
    return np.where(e > 0, y, 0.0)


def hlg_inv(e):
    a, b, c = 0.17883277, 0.28466892, 0.55991073
    x = np.maximum(e, 0.0)
    return np.where(x <= 0.5, x * x / 3.0, (np.exp((x - c) / a) + b) / 12.0)


def curve(tm, x, peak=10.0):
    if tm == 'reinhard':                     # tm_param unset: offset 1
        return x / (x + 1.0) * (peak + 1.0) / peak
    if tm == 'hable':
        def h(v):
            return (v * (v * 0.15 + 0.05) + 0.004) / (v * (v * 0.15 + 0.5) + 0.06) - 0.02 / 0.3
        return h(x) / h(peak)
    j = 0.3                                   # mobius
    a = -j * j * (peak - 1.0) / (j * j - 2.0 * j + peak)
    b = (j * j - 2.0 * j * peak + peak) / max(peak - 1.0, 1e-6)
    return np.where(x <= j, x, (b * b + 2.0 * b * j + j * j) / (b - a) * (x + a) / (x + b))


def tetrahedral(lat, s):
    """lut3d tetrahedral at lattice coordinates s (..., 3) in [0, N-1]: walk
    from the cell's low corner along the axes in decreasing fraction order."""
    n = lat.shape[0]
    base = np.minimum(np.floor(s), n - 2).astype(np.int64)
    d = s - base
    order = np.argsort(-d, axis=-1, kind='stable')
    ds = np.take_along_axis(d, order, axis=-1)
    w = np.stack([1.0 - ds[..., 0], ds[..., 0] - ds[..., 1], ds[..., 1] - ds[..., 2], ds[..., 2]], -1)
    out = np.zeros(s.shape)
    idx = base.copy()
    for k in range(4):
        if k:
            step = np.zeros_like(idx)
            np.put_along_axis(step, order[..., k - 1:k], 1, axis=-1)
            idx = idx + step
        out += w[..., k:k + 1] * lat[idx[..., 2], idx[..., 1], idx[..., 0]]
    return out


def eq_table(gamma, q=8):
    qmax = (1 << q) - 1
    v = np.arange(qmax + 1) / qmax
    t = np.where(v <= 0, 0.0, np.power(np.maximum(v, 1e-300), 1.0 / gamma))
    return np.where(t >= 1.0, qmax, np.floor((qmax + 1) * t)).astype(np.int64)


def rgb_to_xyz(prim, white=(0.3127, 0.3290)):
    """RGB -> XYZ from the primaries' and white's xy chromaticities"""
    P = np.array([[x / y, 1.0, (1 - x - y) / y] for x, y in prim]).T
    wx, wy = white
    Wv = np.array([wx / wy, 1.0, (1 - wx - wy) / wy])
    return P * np.linalg.solve(P, Wv)


def m2020_709():
    """linear BT.2020 -> BT.709 (the LUT-off legacy gamut step, zscale p=bt709)"""
    m2020 = rgb_to_xyz([(0.708, 0.292), (0.170, 0.797), (0.131, 0.046)])
    m709 = rgb_to_xyz([(0.64, 0.33), (0.30, 0.60), (0.15, 0.06)])
    return np.linalg.solve(m709, m2020)


def chain(y, u, v, bits_in, bits_out, hlg, tm, gamma, lut_n, native=False, luma_w=(1.0, 1.0, 1.0)):
    """One frame (planes as integer arrays) -> output planes.  lut_n = 0: the
    LUT off (linear BT.2020 -> BT.709 matrix, BT.1886 encode, clip); native:
    quantise at the output depth (compat8 quantises at 8 bits, then shifts)."""
    s = 1 << (bits_in - 8)
    Y = (y.astype(np.float64) - 16 * s) / (219 * s)
    Cb = upsample((u.astype(np.float64) - 128 * s) / (224 * s))
    Cr = upsample((v.astype(np.float64) - 128 * s) / (224 * s))
    kr, kb = 0.2627, 0.0593
    kg = 1.0 - kr - kb
    E = np.stack([Y + 2 * (1 - kr) * Cr, Y - 2 * kb * (1 - kb) / kg * Cb - 2 * kr * (1 - kr) / kg * Cr,
                  Y + 2 * (1 - kb) * Cb], -1)
    if hlg:
        L = hlg_inv(E)
        ys = L @ np.array([0.2627, 0.6780, 0.0593])
        L = L * (np.where(ys > 0, np.power(np.maximum(ys, 0.0), 0.2), 0.0) * 10.0)[..., None]
    else:
        L = pq_eotf(E) * 100.0
    luma = L @ np.array(luma_w)
    ob = np.maximum(luma - 2.0, 1e-6) / np.maximum(luma, 1e-6)
    L = L * (1 - ob)[..., None] + (luma * ob)[..., None]
    sig = np.maximum(L.max(-1), 1e-6)
    L = L * (curve(tm, sig) / sig)[..., None]
    if lut_n:
        G = np.power(np.maximum(L, 0.0), 1.0 / 2.4)
        rgb = np.clip(tetrahedral(lattice(lut_n), np.clip(G * (lut_n - 1), 0, lut_n - 1)), 0.0, 1.0)
    else:
        rgb = np.clip(np.power(np.maximum(L @ m2020_709().T, 0.0), 1.0 / 2.4), 0.0, 1.0)
    Yo = rgb @ np.array([0.2126, 0.7152, 0.0722])
    cb = (rgb[..., 2] - Yo) / 1.8556
    cr = (rgb[..., 0] - Yo) / 1.5748
    q = bits_out if native else 8
    qs, qmax = float(1 << (q - 8)), (1 << q) - 1
    yq = np.clip(np.floor((16.0 + 219.0 * Yo) * qs + 0.5), 0, qmax).astype(np.int64)
    quad = lambda p: (p[0::2, 0::2] + p[0::2, 1::2] + p[1::2, 0::2] + p[1::2, 1::2]) / 4.0
    cq = [np.clip(np.floor((128.0 + 224.0 * quad(p)) * qs + 0.5), 0, qmax).astype(np.int64) for p in (cb, cr)]
    sh = bits_out - q
    return eq_table(gamma, q)[yq] << sh, cq[0] << sh, cq[1] << sh


CASES = [('hable', 10, 10, False, 2.2, 65), ('reinhard', 10, 8, False, 1.0, 33), ('mobius', 10, 10, False, 1.0, 65),
         ('hable', 12, 12, True, 1.0, 65), ('reinhard', 12, 10, True, 1.6, 17),
         # native quantiser, LUT off (legacy closed form), weighted desat luma (App. B.1 switch)
         ('hable', 10, 10, False, 1.0, 65, 'native'), ('hable', 12, 12, True, 2.2, 65, 'native'),
         ('mobius', 10, 10, False, 2.2, 0), ('hable', 10, 10, False, 1.0, 65, 'bt2020')]


@pytest.mark.parametrize('kind', ['smooth', 'ramp', 'uniform'])
@pytest.mark.parametrize('case', CASES, ids=lambda c: '-'.join(map(str, c)))
def test_independent_restatement_matches_oracle(kind, case):
    tm, bits_in, bits_out, hlg, gamma, lut_n = case[:6]
    native, weighted = 'native' in case[6:], 'bt2020' in case[6:]
    W, H = 96, 64
    fb = synth_frames(kind, 1, W, H, bits_in, device='cpu', seed=11).to_numpy()
    p = oracle.default_params(tonemap=TM[tm], bits_in=bits_in, bits_out=bits_out, transfer_in=1 if hlg else 0,
                              gamma=gamma, mode=1 if native else 0, lut_enabled=1 if lut_n else 0,
                              desat_luma=1 if weighted else 0)
    lat = hdr2sdr.generate_lattice(lut_n) if lut_n else None
    got = hdr2sdr.FrameBatch(oracle.process(p, lat, fb.buf, W, H), W, H, bits_out)
    want = chain(fb.y[0], fb.u[0], fb.v[0], bits_in, bits_out, hlg, tm, gamma, lut_n, native=native,
                 luma_w=(0.2627, 0.6780, 0.0593) if weighted else (1.0, 1.0, 1.0))
    step = 1 << (bits_out - (bits_out if native else 8))
    for name, a, b in zip('YUV', (got.y[0], got.u[0], got.v[0]), want):
        d = np.abs(a.astype(np.int64) - b)
        # eq amplifies a luma flip by the table's slope (<= 256/255 * (1/g) * v^(1/g - 1) steps near black)
        bound = step * (1 if name != 'Y' or gamma == 1.0 else 3)
        assert d.max() <= bound, (name, int(d.max()))
        assert (d > 0).mean() <= 5e-3, (name, float((d > 0).mean()))


# ---- the libplacebo branch (C3, src/utils.py:444-460), max(R,G,B) form ----
def pq_encode(y):
    """ST 2084 inverse EOTF, y = luminance / 10000"""
    m1, m2, c1, c2, c3 = 2610 / 16384, 2523 / 4096 * 128, 3424 / 4096, 2413 / 4096 * 32, 2392 / 4096 * 32
    ym = np.power(np.maximum(y, 0.0), m1)
    return np.power((c1 + c2 * ym) / (1.0 + c3 * ym), m2)


def bt2390(e1, peak_nits=1000.0, white=203.0, knee_offset=1.0):
    """libplacebo bt2390 (PQ in, PQ out) against the SDR target [white/1000,
    white]: Hermite knee at ks = (1 + k) maxLum - k, then the black-point
    lift x += minLum (1 - x)^bp, x = gain (x - minLum) + minLum"""
    lo, hi = pq_encode(0.0), pq_encode(peak_nits / 1e4)
    ml = (pq_encode(white / 1e4) - lo) / (hi - lo)
    mn = (pq_encode(white / 1000.0 / 1e4) - lo) / (hi - lo)
    ks = (1.0 + knee_offset) * ml - knee_offset
    x = np.clip((e1 - lo) / (hi - lo), 0.0, 1.0)
    t = (x - ks) / (1.0 - ks)
    herm = (2 * t ** 3 - 3 * t ** 2 + 1) * ks + (t ** 3 - 2 * t ** 2 + t) * (1 - ks) + (-2 * t ** 3 + 3 * t ** 2) * ml
    x = np.where(x > ks, herm, x)
    bp = min(1.0 / mn, 4.0)
    gain = 1.0 / (1.0 + mn / ml * (1.0 - ml) ** bp)
    x = np.where(x < 1.0, gain * (x + mn * np.power(np.maximum(1.0 - x, 0.0), bp) - mn) + mn, x)
    return x * (hi - lo) + lo


def rgb_to_lms():
    """linear BT.2020 -> LMS (Hunt-Pointer-Estevez rows of XYZ, D65 white)"""
    hpe = np.array([[0.4002, 0.7076, -0.0808], [-0.2263, 1.1653, 0.0457], [0.0, 0.0, 0.9182]])
    return hpe @ rgb_to_xyz([(0.708, 0.292), (0.170, 0.797), (0.131, 0.046)])


def chain_lp(y, u, v, bits_out, lut_n, white=203.0, ipt=False, bits_in=10, hlg=False):
    """PQ 10-bit in; tone curve on max(R,G,B) (or on the intensity of IPT-PQ,
    P and T kept: L'M'S' += I' - I); BT.1886 encode against the
    target black; 8-bit rgba download; lut3d's 8-bit path (truncating);
    BT.709 limited-range Y'CbCr at the output depth, no eq (gamma 1)"""
    s = 1 << (bits_in - 8)
    Y = (y.astype(np.float64) - 16 * s) / (219 * s)
    Cb = upsample((u.astype(np.float64) - 128 * s) / (224 * s))
    Cr = upsample((v.astype(np.float64) - 128 * s) / (224 * s))
    kr, kb = 0.2627, 0.0593
    kg = 1.0 - kr - kb
    E = np.stack([Y + 2 * (1 - kr) * Cr, Y - 2 * kb * (1 - kb) / kg * Cb - 2 * kr * (1 - kr) / kg * Cr,
                  Y + 2 * (1 - kb) * Cb], -1)
    if hlg:                                                  # 1000-nit HLG display (OOTF gamma 1.2)
        L = hlg_inv(E)
        ys = L @ np.array([0.2627, 0.6780, 0.0593])
        L = L * (np.where(ys > 0, np.power(np.maximum(ys, 0.0), 0.2), 0.0) * 1000.0)[..., None]
    else:
        L = pq_eotf(E) * 1e4                                 # nits
    if ipt:
        r2l = rgb_to_lms()
        q = pq_encode(np.minimum(L, 1e8) / 1e4 @ r2l.T)
        I = q @ np.array([0.4, 0.4, 0.2])
        lms = pq_eotf(q + (bt2390(I) - I)[..., None])
        T = lms @ np.linalg.inv(r2l).T * (1e4 / white)
    else:
        sig = np.maximum(L.max(-1), 1e-4)                    # (1e-6 of npl = 100 nits)
        out = pq_eotf(bt2390(pq_encode(sig / 1e4))) * 1e4 / white
        T = L * (out / sig)[..., None]                       # units of the SDR white
    lb = (1.0 / 1000.0) ** (1 / 2.4)
    enc = np.power(np.maximum(T, 0.0) / (1 - lb) ** 2.4, 1 / 2.4) - lb / (1 - lb)
    q8 = np.floor(np.clip(enc, 0.0, 1.0) * 255.0 + 0.5)
    o = tetrahedral(lattice(lut_n), q8 / 255.0 * (lut_n - 1))
    rgb = np.clip(np.floor(o * 255.0), 0, 255) / 255.0
    Yo = rgb @ np.array([0.2126, 0.7152, 0.0722])
    cb = (rgb[..., 2] - Yo) / 1.8556
    cr = (rgb[..., 0] - Yo) / 1.5748
    qs, qmax = float(1 << (bits_out - 8)), (1 << bits_out) - 1
    yq = np.clip(np.floor((16.0 + 219.0 * Yo) * qs + 0.5), 0, qmax).astype(np.int64)
    quad = lambda p: (p[0::2, 0::2] + p[0::2, 1::2] + p[1::2, 0::2] + p[1::2, 1::2]) / 4.0
    cq = [np.clip(np.floor((128.0 + 224.0 * quad(p)) * qs + 0.5), 0, qmax).astype(np.int64) for p in (cb, cr)]
    return yq, cq[0], cq[1]


@pytest.mark.parametrize('kind', ['smooth', 'ramp', 'uniform'])
@pytest.mark.parametrize('bits_in,bits_out,lut_n', [(10, 10, 65), (10, 8, 33), (12, 12, 65)])
@pytest.mark.parametrize('form', ['max-rgb', 'ipt'])
def test_independent_libplacebo_branch_matches_oracle(kind, bits_in, bits_out, lut_n, form):
    """C3's structure (rgba8 download -> lut3d 8-bit -> Y'CbCr at depth) with
    BT.2390 as the max(R,G,B) gain or on the IPT-PQ intensity.  An rgba8 code that rounds the other way
    moves the truncated LUT output by a few 8-bit steps, so a sample may differ
    by up to the lattice's steepest step, and only rarely."""
    W, H = 96, 64
    hlg = bits_in == 12                      # HLG 12-bit input through the same branch
    fb = synth_frames(kind, 1, W, H, bits_in, device='cpu', seed=13).to_numpy()
    p = oracle.default_params(tonemap=7, bits_in=bits_in, bits_out=bits_out, transfer_in=1 if hlg else 0, pipeline=2,
                              lp_tone=1 if form == 'max-rgb' else 0)
    got = hdr2sdr.FrameBatch(oracle.process(p, hdr2sdr.generate_lattice(lut_n), fb.buf, W, H), W, H, bits_out)
    want = chain_lp(fb.y[0], fb.u[0], fb.v[0], bits_out, lut_n, ipt=form == 'ipt', bits_in=bits_in, hlg=hlg)
    k8 = 1 << (bits_out - 8)
    for name, a, b in zip('YUV', (got.y[0], got.u[0], got.v[0]), want):
        d = np.abs(a.astype(np.int64) - b)
        assert d.max() <= 8 * k8, (name, int(d.max()))
        assert (d > 0).mean() <= 1e-2, (name, float((d > 0).mean()))
