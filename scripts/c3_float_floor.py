"""How often do two *exact-arithmetic* float32 implementations of the
libplacebo branch's stage 3 (the IPT-PQ tone form, then the BT.1886 encode
against the target black) round the 8-bit rgba download differently?
(the C3 +-1 step question.)

CPU only (numpy + the C oracle), on a 4K C3 frame (smooth content, and the
reference's website frame).  Variants of the oracle's own chain
(oracle/h2s_oracle.c tone_ipt + lp_encode), each compared with the oracle's
download codes:
  * D  : tone_ipt in float64 (the oracle's statement), restated here in numpy
         -- a check of this restatement (expect 0 flips);
  * Dc : D with the encode's powf correctly rounded (float(pow(double)))
         instead of libm's powf (a 1-ulp-level difference);
  * F  : tone_ipt in float32 throughout (libm powf), i.e. what any faithful
         float32 implementation of the same formula computes.
For each: download codes that differ, and output samples (4:2:0 Y'CbCr at 10
bits after lut3d's 8-bit path) that then differ by more than one step.
Usage: python scripts/c3_float_floor.py [--kind smooth|website]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'hdr-to-sdr_amd'), REPO]
import oracle  # noqa: E402
import hdr2sdr  # noqa: E402
from hdr2sdr.synth import synth_frames, frames_from_rgb8  # noqa: E402

M1, M2, C1, C2, C3 = 0.1593017578125, 78.84375, 0.8359375, 18.8515625, 18.6875


def inv3(m):
    return np.linalg.inv(m)


def ipt_matrices():
    # oracle/h2s_oracle.c ipt_matrices
    xy = np.array([[0.708, 0.292], [0.170, 0.797], [0.131, 0.046], [0.3127, 0.3290]])
    P = np.array([[xy[k, 0] / xy[k, 1] for k in range(3)], [1.0] * 3,
                  [(1 - xy[k, 0] - xy[k, 1]) / xy[k, 1] for k in range(3)]])
    W = np.array([xy[3, 0] / xy[3, 1], 1.0, (1 - xy[3, 0] - xy[3, 1]) / xy[3, 1]])
    S = inv3(P) @ W
    M = P * S[None, :]
    hpe = np.array([[0.4002, 0.7076, -0.0808], [-0.2263, 1.1653, 0.0457], [0.0, 0.0, 0.9182]])
    r2l = hpe @ M
    return r2l, inv3(r2l)


def pq_enc(y, dt):
    y = np.maximum(y, dt(0))
    ym = np.power(y, dt(M1))
    return np.power((dt(C1) + dt(C2) * ym) / (dt(1) + dt(C3) * ym), dt(M2))


def pq_dec(e, dt):
    with np.errstate(invalid='ignore', divide='ignore'):
        xp = np.power(np.maximum(e, dt(0)), dt(1) / dt(M2))
        num = np.maximum(xp - dt(C1), dt(0))
        r = np.power(num / (dt(C2) - dt(C3) * xp), dt(1) / dt(M1))
    return np.where(e > 0, r, dt(0))


def bt2390_consts(peak, tw, tb, knee=1.0):
    smin, smax = float(pq_enc(np.float64(0.0), np.float64)), float(pq_enc(np.float64(peak * 100 / 1e4), np.float64))
    ml = (float(pq_enc(np.float64(tw / 1e4), np.float64)) - smin) / (smax - smin)
    mn = (float(pq_enc(np.float64(tb / 1e4), np.float64)) - smin) / (smax - smin) if tb > 0 else 0.0
    ks = (1 + knee) * ml - knee
    bp = min(1 / mn, 4.0) if mn > 0 else 4.0
    gain = 1 / (1 + mn / ml * (1 - ml) ** bp) if ml < 1 else 1.0
    return dict(smin=smin, smax=smax, ml=ml, mn=mn, ks=ks, bp=bp, gain=gain)


def bt2390_pq_f32(c, e1):
    # oracle bt2390_pq: float arithmetic on a float input
    f = np.float32
    e1 = e1.astype(f)
    e1n = (e1 - f(c['smin'])) / f(c['smax'] - c['smin'])
    e1n = np.clip(e1n, f(0), f(1))
    ks, ml = f(c['ks']), f(c['ml'])
    t = (e1n - ks) / (f(1) - ks)
    t2 = t * t
    t3 = t2 * t
    knee = (f(2) * t3 - f(3) * t2 + f(1)) * ks + (t3 - f(2) * t2 + t) * (f(1) - ks) + (f(-2) * t3 + f(3) * t2) * ml
    e2 = np.where((ks < f(1)) & (e1n > ks), knee, e1n)
    mn = f(c['mn'])
    if c['mn'] > 0:
        lo = e2 < f(1)
        e2b = e2 + mn * np.power(f(1) - e2, f(c['bp']))
        e2b = f(c['gain']) * (e2b - mn) + mn
        e2 = np.where(lo, e2b, e2)
    return e2 * f(c['smax'] - c['smin']) + f(c['smin'])


def tone_ipt(lin, c, r2l, l2r, npl, tw, dt):
    s = dt(npl / 1e4)
    v = np.minimum(lin.astype(dt), dt(1e6)) * s
    q = np.stack([pq_enc(dt(r2l[k, 0]) * v[0] + dt(r2l[k, 1]) * v[1] + dt(r2l[k, 2]) * v[2], dt) for k in range(3)])
    I = dt(0.4) * q[0] + dt(0.4) * q[1] + dt(0.2) * q[2]
    I2 = bt2390_pq_f32(c, I.astype(np.float32)).astype(dt)    # the curve is float in the oracle
    dI = I2 - I
    l = np.stack([pq_dec(q[k] + dI, dt) for k in range(3)])
    os_ = dt(1e4 / tw)
    return np.stack([(dt(l2r[c_, 0]) * l[0] + dt(l2r[c_, 1]) * l[1] + dt(l2r[c_, 2]) * l[2]) * os_
                     for c_ in range(3)]).astype(np.float32)


def lp_encode(x, tw, tb, cr=False):
    lb = (tb / tw) ** (1 / 2.4)
    a, b = np.float32((1 - lb) ** 2.4), np.float32(lb / (1 - lb))
    x = np.where(x > 0, x, np.float32(0)).astype(np.float32)
    y = x / a
    if cr:
        p = np.power(y.astype(np.float64), np.float64(np.float32(1 / 2.4))).astype(np.float32)
    else:
        p = np.power(y, np.float32(1 / 2.4))
    return (p - b).astype(np.float32)


def codes(v):
    v = np.clip(v, np.float32(0), np.float32(1)).astype(np.float32)
    return np.floor(v * np.float32(255) + np.float32(0.5)).astype(np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kind', default='smooth')
    ap.add_argument('--size', default='3840x2160')
    args = ap.parse_args()
    W, H = map(int, args.size.split('x'))
    lat = hdr2sdr.generate_lattice(65)
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
    op = oracle.params_from(params.to_c())
    if args.kind == 'website':
        z = np.load(os.path.join(REPO, 'tests', 'golden', 'website_hdr_full.npz'))
        src = frames_from_rgb8(z[z.files[0]], 1, 10)
        W, H = src.width, src.height
    else:
        src = synth_frames(args.kind, 1, W, H, 10, device='cpu', seed=11)
    buf = src.to_numpy().buf
    lin = oracle.debug_float(op, lat, buf, W, H, 1)
    s2 = oracle.debug_float(op, lat, buf, W, H, 2)
    s3 = oracle.debug_float(op, lat, buf, W, H, 3)
    want = oracle.process(op, lat, buf, W, H).astype(np.int64)
    peak, tw, tb = oracle.resolved(op)[0], 203.0, 0.203
    c = bt2390_consts(peak, tw, tb)
    r2l, l2r = ipt_matrices()
    base = codes(s3)
    out = {'kind': args.kind, 'size': f'{W}x{H}', 'values': int(base.size)}
    d_ipt = tone_ipt(lin, c, r2l, l2r, params.npl, tw, np.float64)
    out['D_stage2_bitexact_share'] = float((d_ipt.view(np.uint32) == s2.view(np.uint32)).mean())
    for name, t2, cr in (('D', d_ipt, False), ('Dc', d_ipt, True),
                         ('F', tone_ipt(lin, c, r2l, l2r, params.npl, tw, np.float32), False)):
        v = lp_encode(t2, tw, tb, cr)
        cd = codes(v)
        flips = cd != base
        rec = {'download_flips': int(flips.sum()), 'flip_share': float(flips.mean()),
               'v_absdiff_codes_p50_p99_max': [float(np.percentile(np.abs(v - s3) * 255, q)) for q in (50, 99, 100)]}
        if flips.any():
            # the output those download codes give: the oracle's downstream (lut3d 8-bit, Y'CbCr) on them
            got = oracle.process_from_rgba8(op, lat, cd.astype(np.uint8), W, H).astype(np.int64) \
                if hasattr(oracle, 'process_from_rgba8') else None
            if got is not None:
                d = np.abs(got - want)
                rec['output_beyond_1_step'] = int((d > 1).sum())
                rec['output_max_diff'] = int(d.max())
        out[name] = rec
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
