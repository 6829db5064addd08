"""Float32 conditioning of the libplacebo branch's IPT tone form (lp_tone
ipt): linear output channel c = sum_k l2r[c, k] LMS_k, so a relative error e
in the LMS values (the PQ EOTF in float32 amplifies one ulp of its pow to
~4e-5) becomes an absolute error up to e sum_k |l2r[c, k]| LMS_k
-- large against a channel the sum cancels to near zero (saturated colours).
Shared by the parity tests and tests/diag/diag_ipt.py."""
import numpy as np


def ipt_matrices():
    """BT.2020 RGB -> LMS (HPE of XYZ, D65) and its inverse, as include/h2s.h
    enum h2s_lp_tone describes them (double)."""
    prim = [(0.708, 0.292), (0.170, 0.797), (0.131, 0.046)]
    wx, wy = 0.3127, 0.3290
    P = np.array([[x / y for x, y in prim], [1.0, 1.0, 1.0], [(1 - x - y) / y for x, y in prim]])
    S = np.linalg.solve(P, np.array([wx / wy, 1.0, (1 - wx - wy) / wy]))
    hpe = np.array([[0.4002, 0.7076, -0.0808], [-0.2263, 1.1653, 0.0457], [0.0, 0.0, 0.9182]])
    r2l = hpe @ (P * S)
    return r2l, np.linalg.inv(r2l)


def ipt_channel_scale(rgb):
    """Per channel, sum_k |l2r[c, k]| |LMS_k| for linear RGB planes [3, H, W]
    (any common unit): the scale the LMS relative error is multiplied by."""
    r2l, l2r = ipt_matrices()
    lms = np.abs(np.einsum('kc,chw->khw', r2l, np.nan_to_num(rgb)))
    return np.einsum('ck,khw->chw', np.abs(l2r), lms)


def lp_encode_spread(params, x, d):
    """Half the spread of the libplacebo branch's BT.1886 encode (against its
    target black) over [x - d, x + d]: the stage-3 image of a stage-2
    uncertainty d (the encode is concave, steepest at 0)."""
    tw = 203.0 if params.target_white is None or params.target_white != params.target_white else params.target_white
    tb = tw / 1000.0 if params.target_black is None or params.target_black != params.target_black else params.target_black
    lb = (tb / tw) ** (1 / 2.4)
    a, b = (1 - lb) ** 2.4, lb / (1 - lb)

    def enc(v):
        return (np.maximum(v, 0.0) / a) ** (1 / 2.4) - b
    x = np.nan_to_num(x)
    return 0.5 * (enc(x + d) - enc(x - d))


def _pq(y):
    m1, m2, c1, c2, c3 = 0.1593017578125, 78.84375, 0.8359375, 18.8515625, 18.6875
    ym = np.maximum(y, 0.0) ** m1
    return ((c1 + c2 * ym) / (1 + c3 * ym)) ** m2


def _eotf(e):
    m1, m2, c1, c2, c3 = 0.1593017578125, 78.84375, 0.8359375, 18.8515625, 18.6875
    xp = np.clip(e, 0.0, 1.0) ** (1 / m2)
    return (np.maximum(xp - c1, 0.0) / (c2 - c3 * xp)) ** (1 / m1)


def ipt_floor(params, lin, want, floor1):
    """The stage-1 absolute uncertainty (floor1, units of npl: a scalar floor,
    or per channel and pixel as stage1_uncertainty gives it) carried through the IPT form to stage 2 (units of the target
    white).  The PQ re-encode of the LMS rows is unboundedly steep at 0, so a
    channel that is nearly black on input can move its L', M' or S' a lot;
    bounded by secants: dq = PQ(y + dy) - PQ(y - dy), the intensity's share
    with the curve's PQ-domain slope taken as <= 1, the EOTF around the output
    L'M'S' and the LMS -> RGB rows' absolute values."""
    r2l, l2r = ipt_matrices()
    npl = params.npl
    tw = 203.0 if params.target_white != params.target_white else params.target_white
    lin = np.nan_to_num(lin)
    y = np.einsum('kc,chw->khw', r2l, lin) * npl / 1e4
    if np.ndim(floor1) == 0:
        dy = (np.abs(r2l).sum(1) * floor1 * npl / 1e4)[:, None, None]
    else:   # per channel and pixel (stage1_uncertainty)
        dy = np.einsum('kc,chw->khw', np.abs(r2l), floor1) * npl / 1e4
    dq = _pq(y + dy) - _pq(np.maximum(y - dy, 0.0))
    d_i = 2.0 * (0.4 * dq[0] + 0.4 * dq[1] + 0.2 * dq[2])
    lp = _pq(np.maximum(np.einsum('kc,chw->khw', r2l, np.nan_to_num(want)) * tw / 1e4, 0.0))
    dl = dq + d_i[None]
    dlms = _eotf(lp + dl) - _eotf(np.maximum(lp - dl, 0.0))
    return np.einsum('ck,khw->chw', np.abs(l2r), dlms) * 1e4 / tw


def pq_eotf_kappa(lin, npl):
    """Condition number |d ln EOTF / d ln E| of the ST 2084 EOTF at the code
    value E that produced each linear value lin (units of npl):
    (1/m1)(1/m2) [xp / (xp - c1) + c3 xp / (c2 - c3 xp)], xp = E^(1/m2).  It
    grows without bound as E falls to c1^m2 (~7.4e-7, EOTF = 0): there any two
    float32 evaluations of the same code differ by kappa times the rounding of
    E itself (about 2^-23 relative), whatever their arithmetic.  0 where lin
    is 0 (both sides read 0 below the pole)."""
    m1, m2, c1, c2, c3 = 0.1593017578125, 78.84375, 0.8359375, 18.8515625, 18.6875
    y = np.nan_to_num(np.abs(lin), nan=0.0, posinf=0.0) * npl / 1e4
    e = _pq(y)
    xp = np.clip(e, 0.0, None) ** (1 / m2)
    with np.errstate(divide='ignore', invalid='ignore'):
        k = (1 / m1) * (1 / m2) * (xp / (xp - c1) + c3 * xp / (c2 - c3 * xp))
    return np.where(y > 0, np.nan_to_num(np.abs(k), nan=0.0, posinf=0.0), 0.0)


def stage1_uncertainty(lin, npl, transfer):
    """Absolute stage-1 uncertainty (units of npl, per channel and pixel)
    that conditioning alone puts between any two float32 evaluations of the
    EOTF of the same code, with no floor: the PQ EOTF's kappa times the
    relative disagreement of its inputs -- E itself, a sum of O(1) float32
    terms (Y' and the chroma products: 2^-22 absolute between two
    evaluations, so 2^-22 / E relative, large where the terms cancel to a
    near-black channel), and E^(1/m2), whose 2-ulp disagreement (2^-22)
    enters the EOTF m2-fold through kappa.  HLG (transfer 'arib-std-b67'):
    below E = 1/2 the inverse OETF is E^2 / 3 and the OOTF raises it to 1.2,
    so the same 2^-22 absolute in E is 2.4 x 2^-22 / E relative, E estimated
    back from the display value (1000-nit peak)."""
    a = np.nan_to_num(np.abs(lin), nan=0.0, posinf=0.0)
    if transfer not in ('smpte2084', 'pq'):
        # display -> scene light per channel: Fd = 1000 Ys^0.2 Fs (units of
        # nits), Ys the scene luminance (BT.2100 OOTF)
        yd = np.einsum('c,chw->hw', np.array([0.2627, 0.6780, 0.0593]), a) * npl / 1000.0
        ys = yd ** (1 / 1.2)
        with np.errstate(divide='ignore', invalid='ignore'):
            fs = np.where(ys > 0, a * npl / 1000.0 / ys[None] ** 0.2, 0.0)
        e = np.sqrt(3.0 * np.minimum(fs, 1.0 / 12))          # the square-law branch
        with np.errstate(divide='ignore', invalid='ignore'):
            rel = np.where(e > 0, 2.4 * 2.0 ** -22 / e, 0.0)
        return (rel + 2.0 ** -22) * a
    m2 = 78.84375
    kap = pq_eotf_kappa(lin, npl)
    e = _pq(a * npl / 1e4)
    with np.errstate(divide='ignore', invalid='ignore'):
        rel = np.where(e > 0, 2.0 ** -22 / e, 0.0)
    return kap * (rel + m2 * 2.0 ** -22) * a
