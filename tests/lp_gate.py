"""The libplacebo branch's integer gate: per-sample
attribution of every output sample that sits more than one step from the
oracle, instead of round 5's blanket "k8 steps on up to 0.3 % of samples".

The branch downloads its BT.1886-encoded R'G'B' as 8-bit rgba codes
(`libplacebo=...:format=rgba,hwdownload,format=rgba`, src/utils.py:444-460)
and lut3d's 8-bit path then truncates its output to 8 bits, so a download
code that rounds the other way moves the output by up to k8 lattice steps.
The reference computes the download in libplacebo's float32 GLSL, so no
float32 evaluation is "the" reference: the oracle states stages 1-3 as exact
(double) arithmetic (oracle/h2s_oracle.c chain_lp_d) and exports the exact
pre-rounding value x of each download channel (oracle.lp_download; the code
is floor(x)).  A float32 kernel lands within its own stated error bound of x
(float_gate.lp_stage3_bound: the float gate's conditioning model at stage 3
plus the encode's rounding), so it can round a channel the other way only
where x lies within that bound of an integer.

The gate, per output sample beyond one quantiser step (luma judged before eq,
as the CPU chain's gate does; chroma as quantiser codes):
* it is ATTRIBUTED if some download channel of a pixel it depends on (luma:
  the pixel; chroma: the 2 x 2 quad, or the bicubic decimation's 7 x 8
  support) lies within the kernel's bound of a rounding boundary;
* every other beyond sample is UNATTRIBUTED, and there must be none;
* attributed samples stay within the k8 lattice bound.
Pure: numpy in, a report out (tests/test_lp_gate.py runs it on the oracle's
own float32 form and on a one-code stage-3 bias, on the CPU).
"""
import math

import numpy as np

import oracle
from float_gate import Planes, lattice_max_step, lp_stage3_bound


def _eq_window(op, q, want_q):
    """Luma after eq: the codes eq[q0 - 1] .. eq[q1 + 1] around the oracle's
    pre-eq code range (as test_gpu_parity.assert_close_int)."""
    eq = oracle.resolved(op)[2].astype(np.int64)
    lo_i = np.searchsorted(eq, want_q, side='left')
    hi_i = np.searchsorted(eq, want_q, side='right') - 1
    return eq[np.clip(lo_i - 1, 0, len(eq) - 1)], eq[np.clip(hi_i + 1, 0, len(eq) - 1)]


def beyond_samples(params, got, want, W, H):
    """(luma mask [F, H, W], chroma mask [F, H/2, W/2], step): the samples
    beyond one quantiser step of the oracle."""
    op = oracle.params_from(params.to_c())
    q = oracle.quant_bits(op)
    shift = max(0, params.bits_out - q)
    F, ysz = got.shape[0], W * H
    gy, wy = got[:, :ysz] >> shift, want[:, :ysz] >> shift
    if params.gamma == 1.0:
        by = np.abs(gy - wy) > 1
    else:
        lo, hi = _eq_window(op, q, wy)
        by = (gy < lo) | (gy > hi)
    gc, wc = got[:, ysz:] >> shift, want[:, ysz:] >> shift
    bc = (np.abs(gc - wc) > 1).reshape(F, 2, H // 2, W // 2).any(axis=1)
    return by.reshape(F, H, W), bc, 1 << shift


def _offsets(params):
    """Luma offsets (dy, dx) from (2 cy, 2 cx) that a chroma sample reads:
    the 2 x 2 quad (box), or the bicubic decimation's 8 rows x 7 columns."""
    if params.chroma_filter == 'bicubic':
        return [(dy, dx) for dy in range(-3, 5) for dx in range(-3, 4)]
    return [(0, 0), (0, 1), (1, 0), (1, 1)]


def _support(params, bc, W, H):
    """Luma pixels the chroma samples in bc [H/2, W/2] depend on."""
    m = np.zeros((H, W), bool)
    cy, cx = np.nonzero(bc)
    for dy, dx in _offsets(params):
        m[np.clip(2 * cy + dy, 0, H - 1), np.clip(2 * cx + dx, 0, W - 1)] = True
    return m


def _chroma_any(params, tie, W, H):
    """[H/2, W/2]: some pixel a chroma sample reads is in tie [H, W] (edge-clamped)."""
    cy, cx = np.mgrid[0:H // 2, 0:W // 2]
    out = np.zeros((H // 2, W // 2), bool)
    for dy, dx in _offsets(params):
        out |= tie[np.clip(2 * cy + dy, 0, H - 1), np.clip(2 * cx + dx, 0, W - 1)]
    return out


def attribute(params, kernel, got, want, src, W, H, lut_n=65, lattice=None, knees=None):
    """Attribute every beyond-one-step sample of got (vs the oracle's want,
    both [F, W*H*3/2] int64) to a download near-tie within the kernel's
    bound.  src: the input batch (host numpy, [F, ...]).  knees: under
    dynamic peak detection, each frame's (peak, average PQ) as
    oracle.process_dynamic(knees=...) reports them.  Returns a report:
    samples, beyond, attributed, unattributed (counts), max_steps, k8_steps,
    near_tie_px (pixels examined that had a channel within the bound)."""
    from float_gate import lattice as _lat
    lat = _lat(lut_n) if lattice is None else lattice
    by, bc, step = beyond_samples(params, got, want, W, H)
    k8 = math.ceil(lattice_max_step(lut_n) * (lut_n - 1)) + 1
    op = oracle.params_from(params.to_c())
    q = oracle.quant_bits(op)
    rep = dict(samples=int(got.size), beyond=int(by.sum() + bc.sum()), attributed=0, unattributed=0,
               max_steps=int(-(-int(np.abs(got - want).max(initial=0)) // step)), k8_steps=k8,
               k8_bound_out_steps=math.ceil(k8 * 224 * (1 << (q - 8)) / 255) + 1, near_tie_px=0,
               unattributed_where=[])
    if rep['beyond'] == 0:
        return rep
    qs = 219.0 if params.lp_range == 'limited' else 255.0
    for f in range(got.shape[0]):
        if not (by[f].any() or bc[f].any()):
            continue
        one = np.ascontiguousarray(src[f:f + 1])
        pf, avg = params, 0.0
        if knees is not None:      # this frame's detected peak and knee, as static parameters
            pf, avg = params.with_(peak=knees[f][0], peak_detect=False), knees[f][1]
        opf = oracle.params_from(pf.to_c())
        P = Planes(pf, one, W, H, lut_n, avg_pq=avg)
        xq = oracle.lp_download(opf, lat, one, W, H, avg_pq=avg)  # [3, H, W] exact pre-rounding values
        need = by[f] | _support(params, bc[f], W, H)
        ys, xs = np.nonzero(need)
        bound = lp_stage3_bound(pf, kernel, P, ys, xs) * qs      # codes
        x = xq[:, ys, xs]
        near = (np.abs(x - np.round(x)) <= bound).any(axis=0)
        tie = np.zeros((H, W), bool)
        tie[ys[near], xs[near]] = True
        rep['near_tie_px'] += int(near.sum())
        # luma: the pixel itself
        ly, lx = np.nonzero(by[f])
        ok_y = tie[ly, lx]
        # chroma: any pixel of its support
        cy, cx = np.nonzero(bc[f])
        ok_c = _chroma_any(params, tie, W, H)[cy, cx]
        rep['attributed'] += int(ok_y.sum() + ok_c.sum())
        bad = int((~ok_y).sum() + (~ok_c).sum())
        rep['unattributed'] += bad
        if bad and len(rep['unattributed_where']) < 8:
            for a, b in list(zip(ly[~ok_y], lx[~ok_y]))[:4]:
                rep['unattributed_where'].append(('Y', f, int(a), int(b)))
            for a, b in list(zip(cy[~ok_c], cx[~ok_c]))[:4]:
                rep['unattributed_where'].append(('C', f, int(a), int(b)))
    return rep


def check(params, kernel, got, want, src, W, H, lut_n=65, max_attributed_frac=3e-3, knees=None):
    """The gate as failures (empty list = pass)."""
    rep = attribute(params, kernel, got, want, src, W, H, lut_n, knees=knees)
    fails = []
    if rep['unattributed']:
        fails.append(f"{rep['unattributed']} samples beyond one step with no download channel within the "
                     f"{kernel} bound of a rounding tie (first: {rep['unattributed_where'][:4]})")
    if rep['max_steps'] > rep['k8_bound_out_steps']:
        fails.append(f"max diff {rep['max_steps']} output steps > the k8 bound {rep['k8_bound_out_steps']}")
    if rep['attributed'] > max_attributed_frac * rep['samples']:
        fails.append(f"{rep['attributed']} attributed samples > {max_attributed_frac:.2%} of {rep['samples']}")
    return rep, fails
