"""How often does a table-driven float32 IPT form round the libplacebo
branch's 8-bit rgba download differently from the oracle, as a function of
the PQ-encode table's resolution?  (cut the IPT table
error.)  CPU only: the IPT form restated with the tile kernel's tables
(cubic segments through Chebyshev nodes, float32 coefficients and Horner
evaluation; PQ encode per octave from 2^-34 with the direct form below; PQ
EOTF at 128 segments per unit), the oracle's own curve and encode
(scripts/c3_float_floor.py), against the oracle's download codes on a smooth
C3 frame.  Round 5, 1920x1080 smooth: 4 segments per octave 3,275 flips
(0.053 %), 8: 473 (0.008 %), 16: 432 -- the float32 floor of the form; the
EOTF table's resolution does not matter.  Usage:
python scripts/c3_table_flips.py [--size WxH]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c3_float_floor import (bt2390_consts, bt2390_pq_f32, codes, hdr2sdr, ipt_matrices, lp_encode,  # noqa: E402
                            oracle, pq_dec, pq_enc, synth_frames)

f32 = np.float32
NODES = (1 - np.cos((2 * np.arange(4) + 1) * np.pi / 8)) / 2


def horner(C, idx, t):
    c = C[idx]
    r = (c[:, 3].astype(np.float64) * t + c[:, 2]).astype(f32)
    r = (r.astype(np.float64) * t + c[:, 1]).astype(f32)
    return (r.astype(np.float64) * t + c[:, 0]).astype(f32)


def pqi_table(per_oct, oct0=-34, top=14):
    A = np.vander(NODES / per_oct, 4, increasing=True)
    n = (top - oct0) * per_oct
    C = np.zeros((n, 4))
    for sg in range(n):
        base = 2.0 ** (oct0 + sg // per_oct)
        C[sg] = np.linalg.solve(A, pq_enc(base * (1 + (sg % per_oct) / per_oct + NODES / per_oct), np.float64))
    return C.astype(f32)


def pqi_eval(C, y, per_oct, oct0=-34):
    y = np.maximum(y.astype(f32), f32(0))
    b = y.view(np.uint32)
    sh = 23 - int(np.log2(per_oct))
    sr = (b >> sh).astype(np.int64) - (127 + oct0) * per_oct
    t = ((b & np.uint32((1 << sh) - 1)) | np.uint32(0x3f800000)).view(f32) - f32(1)
    v = horner(C, np.clip(sr, 0, len(C) - 1), t)
    low = sr < 0
    v[low] = pq_enc(y[low], f32)
    return v


def pqz_table(seg=128, nseg=240):
    A = np.vander(NODES, 4, increasing=True)
    C = np.stack([np.linalg.solve(A, pq_dec((i + NODES) / seg, np.float64)) for i in range(nseg)])
    C[0, 0] = 0
    return C.astype(f32)


def pqz_eval(C, e, seg=128):
    u = (np.clip(e, 0, 1.87).astype(np.float64) * seg).astype(f32)
    i = np.floor(u)
    return horner(C, np.clip(i.astype(np.int64), 0, len(C) - 1), (u - i).astype(f32))


def tone_tab(lin, c, r2l, l2r, npl, tw, per_oct):
    Cq, Cz = pqi_table(per_oct), pqz_table()
    v = np.minimum(lin.astype(f32), f32(1e6)) * f32(npl / 1e4)
    shp = v.shape[1:]
    q = np.stack([pqi_eval(Cq, (f32(r2l[k, 0]) * v[0] + f32(r2l[k, 1]) * v[1] + f32(r2l[k, 2]) * v[2]).ravel(),
                           per_oct).reshape(shp) for k in range(3)])
    I = f32(0.4) * q[0] + f32(0.4) * q[1] + f32(0.2) * q[2]
    dI = bt2390_pq_f32(c, I) - I
    l = np.stack([pqz_eval(Cz, (q[k] + dI).ravel()).reshape(shp) for k in range(3)])
    return np.stack([(f32(l2r[j, 0]) * l[0] + f32(l2r[j, 1]) * l[1] + f32(l2r[j, 2]) * l[2]) * f32(1e4 / tw)
                     for j in range(3)]).astype(f32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--size', default='1920x1080')
    W, H = map(int, ap.parse_args().size.split('x'))
    lat = hdr2sdr.generate_lattice(65)
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
    op = oracle.params_from(params.to_c())
    buf = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=11).to_numpy().buf
    lin = oracle.debug_float(op, lat, buf, W, H, 1)
    s3 = oracle.debug_float(op, lat, buf, W, H, 3)
    peak, tw, tb = oracle.resolved(op)[0], 203.0, 0.203
    c = bt2390_consts(peak, tw, tb)
    r2l, l2r = ipt_matrices()
    base = codes(s3)
    out = {'size': f'{W}x{H}', 'values': int(base.size)}
    for per_oct in (4, 8, 16):
        with np.errstate(all='ignore'):
            v = lp_encode(tone_tab(lin, c, r2l, l2r, params.npl, tw, per_oct), tw, tb, True)
        flips = codes(v) != base
        out[f'pqi_{per_oct}_per_octave'] = {
            'download_flips': int(flips.sum()), 'flip_share': float(flips.mean()),
            'dv_codes_p50_p99': [float(np.percentile(np.abs(v - s3) * 255, q)) for q in (50, 99)]}
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
