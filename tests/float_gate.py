"""The 1e-3 float gate of north_star ("within 1e-3 relative on the
intermediate float path") as pure functions of the oracle's planes, so that
the same gate judges the GPU kernels' debug planes (tests/test_gpu_parity.py
check_float_stage, -m gpu) and, on the CPU, mutated copies of the oracle's own
planes (tests/test_float_gate.py): a gate that accepts the exact oracle must
reject a 2e-3 error on one value and a 1.2e-3 error on 1 % of them
(VERDICT r04 item 2).

What is allowed beyond 1e-3 relative, and why:
* the EOTF's own conditioning at stage 1 (kappa times the disagreement any two
  float32 evaluations of the same code have; tests/ipt_cond.py
  stage1_uncertainty), carried through the tone gain at stage 2, through
  x^(1/2.4) at stage 3 and through the lattice's local slope at stages 4/5;
* vf_tonemap's desaturation threshold (kappa = luma / (luma - desat)), and
  Hable's cancellation next to black (tone_uncertainty);
* the IPT form's LMS -> RGB rows on the libplacebo branch (EPS_IPT);
* floors at stages 3/4 (1e-5) and 5 (224 2^(q-8) 1e-5), where values near 0
  in gamma space have no relative scale;
* after the libplacebo branch's 8-bit download (stages 4/5): a pixel whose
  download rounded the other way, only if the oracle's stage-3 value of one
  of its channels lies within TIE_WINDOW codes of the download's rounding
  boundary (the flips' measured window), within the lattice's k8 bound;
* excluded and counted: pixels past the ST 2084 pole (linear > 1e6 npl) and
  at vf_tonemap's desat kink (kappa > 50).
"""
import math

import numpy as np

import oracle
import hdr2sdr

FLOAT_CFGS = {
    'C2_hable_pq10': dict(tonemapper='hable', gamma=2.2, bits_out=10),
    'C3_bt2390_pq10_cpu': dict(tonemapper='bt.2390', pipeline='cpu', bits_out=10),
    'C5_hable_hlg12': dict(tonemapper='hable', bits_in=12, bits_out=12, transfer='arib-std-b67'),
    'C4_mobius_native': dict(tonemapper='mobius', bits_out=10, mode='native'),
    # the libplacebo branch (the reference's C3 chain, src/utils.py:444-460):
    # knee offset 1.0, black point 0.203 nits, target white 203, rgba8 + lut3d 8-bit
    # (tone curve on the IPT-PQ intensity, the default; and the max(R,G,B) gain)
    'C3_bt2390_libplacebo': dict(tonemapper='bt.2390', bits_out=10),
    'C3_bt2390_libplacebo_max_rgb': dict(tonemapper='bt.2390', bits_out=10, lp_tone='max-rgb'),
    'spline_libplacebo_hlg12': dict(tonemapper='spline', bits_in=12, bits_out=12, transfer='arib-std-b67'),
    'C3_bt2390_libplacebo_lut_off': dict(tonemapper='bt.2390', bits_out=10, lut_enabled=False),
    'hable_libplacebo': dict(tonemapper='hable', bits_out=10, pipeline='libplacebo'),
}

# share of kept values that fail 1e-3 relative and pass only through a floor
# or conditioning term, per content (the report's floor_only_frac)
FLOOR_ONLY_MAX = {'ramp': 0.06, 'edges': 0.05, 'uniform': 0.03, 'smooth': 0.02}
TILE_DARK_EXACT = True    # k_tile evaluates its PQ table's first segment exactly (h2s_tile.h dark re-run): no table floor
EPS_IPT = 2e-5            # LMS relative error of the IPT form on the tile kernel (tests/diag/diag_ipt.py: max 1.33e-5, round 5)
TIE_WINDOW = 0.25         # download codes: a flip must sit this close to the rounding boundary (measured max 0.16)

_LAT = {}


def lattice(n):
    if n not in _LAT:
        _LAT[n] = hdr2sdr.generate_lattice(n)
    return _LAT[n]


def lattice_max_step(n):
    a = lattice(n).reshape(n, n, n, 3).astype(np.float64)
    return max(float(np.abs(np.diff(a, axis=ax)).max()) for ax in range(3))


def lattice_slope(n, s3):
    """Per pixel, output channel and input axis: the largest |corner
    difference| along that axis over the lattice cell that holds the stage-3
    coordinates s3 (3, H, W) in [0, 1], times (n - 1): a bound on the
    tetrahedral interpolant's partial derivatives there (it is linear on each
    tetrahedron, with slopes equal to corner differences).  Returns (c, a, H, W)."""
    a = lattice(n).reshape(n, n, n, 3).astype(np.float64)          # [b][g][r][c]
    x = np.clip(np.nan_to_num(s3, nan=0.0), 0.0, 1.0) * (n - 1)
    i = np.minimum(np.floor(x).astype(np.int64), n - 2)
    ir, ig, ib = i[0], i[1], i[2]
    out = np.zeros((3, 3) + s3.shape[1:])
    for ax in range(3):          # 0 = r, 1 = g, 2 = b
        best = np.zeros((3,) + s3.shape[1:])
        for db in (0, 1):
            for dg in (0, 1):
                for dr in (0, 1):
                    if (dr, dg, db)[ax]:
                        continue
                    lo = a[ib + db, ig + dg, ir + dr]
                    hi = a[ib + db + (ax == 2), ig + dg + (ax == 1), ir + dr + (ax == 0)]
                    best = np.maximum(best, np.moveaxis(np.abs(hi - lo), -1, 0))
        out[:, ax] = best * (n - 1)
    return out


def tone_uncertainty(params, op):
    """Absolute stage-2 uncertainty (units of the curve's output white) of a
    tone curve whose float32 form cancels next to black: Hable's
    (x(Ax+CB)+DE)/(x(Ax+B)+DF) - E/F subtracts two values near E/F = 0.067,
    so any two float32 evaluations differ by a few ulp of E/F, 2^-21 E/F,
    divided by the normalisation hable(peak) -- 2 % of a 4e-7 output.  Both
    vf_tonemap's form and libplacebo's (NORM scaling: the source peak over the
    SDR white) have it; 0 for the other curves."""
    if params.tonemapper != 'hable':
        return 0.0
    A, B, C, D, E, F = 0.15, 0.50, 0.10, 0.20, 0.02, 0.30

    def hable(x):
        return (x * (A * x + C * B) + D * E) / (x * (A * x + B) + D * F) - E / F
    if params.resolved_pipeline() == 'libplacebo':
        peak = oracle.resolved(op)[0] * params.npl / 203.0    # source peak over the SDR white (lp NORM)
    else:
        peak = oracle.resolved(op)[0]
    return 2.0 ** -21 * (E / F) / hable(max(peak, 1.0))


class Planes:
    """The oracle's float planes of one frame (stages 1..5, computed on demand)."""

    def __init__(self, params, buf, W, H, lut_n=65, avg_pq=0.0):
        self.params, self.buf, self.W, self.H, self.lut_n, self.avg_pq = params, buf, W, H, lut_n, avg_pq
        self.op = oracle.params_from(params.to_c())
        self._p = {}

    def __getitem__(self, stage):
        if stage not in self._p:
            self._p[stage] = oracle.debug_float(self.op, lattice(self.lut_n), self.buf, self.W, self.H,
                                                stage, avg_pq=self.avg_pq).astype(np.float64)
        return self._p[stage]


class Tolerance:
    pass


def _stage2_spread(params, P, U1, lin=None):
    """sum_k |J[c, k]| U1[k]: the stage-1 uncertainty U1 (3, H, W) carried
    through the chain's tone map, J its Jacobian at the oracle's stage-1
    values by central differences of the oracle's own S2 (oracle.tonemap_lin;
    steps of 1e-3 relative, so float32 noise stays far below the tolerance).
    This is what desaturation's luma mixing (kappa), the tone gain and, on
    the libplacebo branch, the IPT rows and the black-point lift do to an
    input disagreement -- per channel, not the pixel's largest channel.
    lin: the stage-1 values to take it at (any (3, ...) subset of P[1])."""
    lin = np.nan_to_num(P[1] if lin is None else lin, nan=0.0, posinf=0.0).astype(np.float64)
    out = np.zeros(lin.shape)
    lat = lattice(P.lut_n) if params.lut_enabled else None
    for k in range(3):
        h = np.maximum(1e-3 * np.abs(lin[k]), 1e-9)
        hi, lo = lin.copy(), lin.copy()
        hi[k] += h
        lo[k] = np.maximum(lin[k] - h, 0.0)
        fh = oracle.tonemap_lin(P.op, lat, hi.astype(np.float32), avg_pq=P.avg_pq).astype(np.float64)
        fl = oracle.tonemap_lin(P.op, lat, lo.astype(np.float32), avg_pq=P.avg_pq).astype(np.float64)
        with np.errstate(invalid='ignore'):
            J = np.nan_to_num((fh - fl) / (hi[k] - lo[k])[None], nan=0.0, posinf=0.0, neginf=0.0)
        out += np.abs(J) * U1[k][None]
    return out


def lp_stage3_bound(params, kernel, P, ys, xs):
    """The stated error bound of a kernel's libplacebo-branch stage-3 value
    (the BT.1886-encoded R'G'B' the 8-bit rgba download rounds), per channel
    at the pixels (ys, xs) of P's frame, in units of that value ([0, 1]):
    the float gate's own propagation (float_tolerance's U at stage 3 -- the
    EOTF's conditioning at stage 1 carried through the tone map's Jacobian,
    the tone curve's cancellation, on k_tile's IPT form EPS_IPT through the
    LMS -> RGB rows, then the encode's slope) plus the float32 encode's own
    rounding (v_log_f32 / v_exp_f32 or powf: a few ulp of the exponent
    log2(x) / 2.4 and of the result).  kernel: 'k_tile', 'generic' (a float32
    restatement: the round-5 oracle form), or 'exact' (double arithmetic:
    the generic kernel's libplacebo path, H2S_OPT_LP_EXACT).  Returns (3, n)."""
    from ipt_cond import ipt_channel_scale, lp_encode_spread, stage1_uncertainty
    n = len(ys)
    t2 = np.nan_to_num(P[2][:, ys, xs]).reshape(3, 1, n)
    t3 = np.nan_to_num(P[3][:, ys, xs]).reshape(3, 1, n)
    if kernel == 'exact':
        return (1e-12 * (1.0 + np.abs(t3))).reshape(3, n)
    lin = np.nan_to_num(P[1][:, ys, xs], nan=0.0, posinf=0.0).reshape(3, 1, n)
    # stage1_uncertainty / tone_uncertainty bound the disagreement of TWO
    # float32 evaluations; against exact arithmetic a float32 kernel carries
    # one of them: half
    U = 0.5 * stage1_uncertainty(lin, params.npl, params.transfer)
    U = _stage2_spread(params, P, U, lin=lin) + 0.5 * tone_uncertainty(params, P.op)
    if kernel == 'k_tile' and params.lp_tone == 'ipt':
        U = U + EPS_IPT * ipt_channel_scale(t2)
    if params.lp_tone == 'max-rgb' and params.tonemapper in ('bt.2390', 'spline'):
        # the gain's own EOTF: s2 = EOTF(curve(PQ(sig))) is a second float32
        # decode, with the EOTF's conditioning at the curve's output (the
        # stage-1 model at s2), scaling every channel alike (c s2 / sig)
        tw_ = 203.0 if params.target_white != params.target_white else params.target_white
        s2 = np.max(np.abs(t2), axis=0, keepdims=True) * tw_ / params.npl      # units of npl
        with np.errstate(divide='ignore', invalid='ignore'):
            rel = np.nan_to_num(0.5 * stage1_uncertainty(np.repeat(s2, 3, axis=0), params.npl, 'pq')[:1] / s2,
                                nan=0.0, posinf=0.0)
        U = U + rel * np.abs(t2)
    U3 = lp_encode_spread(params, t2, U)
    tw = 203.0 if params.target_white != params.target_white else params.target_white
    tb = tw / 1000.0 if params.target_black != params.target_black else params.target_black
    lb = (tb / tw) ** (1 / 2.4)
    a, b = (1 - lb) ** 2.4, lb / (1 - lb)
    with np.errstate(divide='ignore', invalid='ignore'):
        l2 = np.abs(np.nan_to_num(np.log2(np.maximum(t2, 1e-30) / a), posinf=0.0, neginf=0.0))
    enc = 2.0 ** -21 * (np.abs(t3) + b) * (1.0 + l2)
    return np.nan_to_num(U3 + enc, nan=0.0, posinf=0.0).reshape(3, n)


def float_tolerance(params, kernel, stage, kind, P):
    """Per-value tolerance of the (kernel, stage) float check on the oracle's
    planes P (a Planes); pure: depends on the oracle only.  tol = 1e-3
    relative + U, U the uncertainty the chain's own conditioning puts on the
    stage (stage 1: the EOTF's kappa, and k_tile's first-segment table floor;
    carried stage to stage by the Jacobian of the tone map, the derivative of
    the encode and the lattice's local slope) + the stage floor.  Returns a
    Tolerance with want (the stage plane, as the kernel reports it), tol,
    rel (the 1e-3 part), floor, keep (not excluded), skip (excluded pixels),
    seg0 and near_tie (libplacebo branch, stage >= 4)."""
    from ipt_cond import stage1_uncertainty
    op = P.op
    T = Tolerance()
    want = P[stage].copy()
    if stage == 3 and kernel == 'k_tile':
        want = np.clip(want, 0.0, 1.0)      # k_tile clamps x to [0, 1) before the power (lattice coordinate)
    q = oracle.quant_bits(op)
    T.q = q
    lp = params.resolved_pipeline() == 'libplacebo'
    # floors: none at stages 1/2 (conditioning only), 1e-5 at 3/4, 224 2^(q-8)
    # 1e-5 at 5 (code units at depth q)
    floor = {1: 0.0, 2: 0.0, 3: 1e-5, 4: 1e-5, 5: 224 * (1 << (q - 8)) * 1e-5}[stage]
    lin = P[1]
    skip = ~(np.nanmax(np.abs(np.nan_to_num(lin, nan=np.inf)), axis=0) < 1e6)
    U = stage1_uncertainty(lin, params.npl, params.transfer)
    # k_tile's PQ table's first segment (E < 1/128, below 0.0015 nits): its
    # cubic holds 7.3e-8 x npl absolute, not 1e-3 relative, unless the build
    # evaluates that segment exactly (TILE_DARK_EXACT)
    seg0 = np.zeros(lin.shape, bool)
    if kernel == 'k_tile' and not TILE_DARK_EXACT and params.transfer in ('smpte2084', 'pq'):
        seg0 = np.nan_to_num(lin, nan=np.inf) < oracle.pq_eotf(1.0 / 128) * 1e4 / params.npl
        U = U + np.where(seg0, 2e-7, 0.0)
    kappa = np.zeros(skip.shape)
    if stage >= 2 and params.desat > 0 and params.tonemapper not in ('bt.2390', 'spline') and not lp:
        # vf_tonemap's desat kink: excluded where kappa = luma / (luma - desat)
        # > 50 (the tone map is not differentiable there)
        wts = {'rgb': (1, 1, 1), 'bt2020': (0.2627, 0.6780, 0.0593), 'bt709': (0.2126, 0.7152, 0.0722)}
        lr, lg, lb = wts[params.desat_luma]
        with np.errstate(invalid='ignore', divide='ignore'):
            luma = lr * lin[0] + lg * lin[1] + lb * lin[2]
            skip |= np.abs(luma - params.desat) < 0.02 * luma
            kappa = np.nan_to_num(np.where(luma > params.desat, luma / (luma - params.desat), 0.0),
                                  nan=0.0, posinf=0.0)
    keep = np.broadcast_to(~skip[None], want.shape)
    if stage >= 2:
        U = _stage2_spread(params, P, U) + tone_uncertainty(params, op)
        if kernel == 'k_tile' and lp and params.lp_tone == 'ipt':
            # the tile kernel's IPT form reads its PQ encode / EOTF tables: LMS
            # relative error <= EPS_IPT, through the LMS -> RGB rows
            from ipt_cond import ipt_channel_scale
            U = U + EPS_IPT * ipt_channel_scale(P[2])
    if stage >= 3:
        w2 = np.nan_to_num(P[2])
        if lp:
            from ipt_cond import lp_encode_spread
            if not params.lut_enabled:      # LUT off: the BT.2020 -> 709 matrix first
                m709 = np.array(oracle.BT2020_TO_BT709)
                w2, U = np.einsum('ck,khw->chw', m709, w2), np.einsum('ck,khw->chw', np.abs(m709), U)
            U = lp_encode_spread(params, w2, U)
        else:                               # x^(1/2.4), by secants (steep at 0)
            def g(x):
                return np.maximum(x, 0.0) ** (1 / 2.4)
            U = 0.5 * (g(w2 + U) - g(w2 - U))
    if stage >= 4 and not lp and params.lut_enabled:   # the tetrahedral interpolant's local slope
        U = np.einsum('cahw,ahw->chw', lattice_slope(P.lut_n, P[3]), U + 1e-5)
    if lp and params.lut_enabled and stage >= 4:
        # after the 8-bit download the values are exact functions of the
        # download codes: equal codes give equal values (float noise), a code
        # that rounded the other way is judged by the near-tie rule below
        U = np.zeros(want.shape)
    if stage == 5:            # the Y'CbCr rows at the quantiser's scale (|row| sums <= 1)
        U = 224 * (1 << (q - 8)) * U.max(axis=0, keepdims=True)
    rel = 1e-3 * np.abs(want)
    tol = rel + floor + np.nan_to_num(U, nan=0.0)
    T.near_tie = None
    if lp and params.lut_enabled and stage >= 4:
        # the download's rounding boundary: code = floor(v qs + qo + 0.5);
        # distance of the oracle's stage-3 value (in codes) to it, per pixel
        lim = params.lp_range == 'limited'
        qs, qo = (219.0, 16.0) if lim else (255.0, 0.0)
        x = np.clip(np.nan_to_num(P[3]), 0.0, 1.0) * qs + qo + 0.5
        dist = np.abs(x - np.round(x))
        T.near_tie = (dist < TIE_WINDOW).any(axis=0)
        k8 = math.ceil(lattice_max_step(65) * 64) + 1
        T.flip_lim = k8 / 255.0 if stage == 4 else 224 * (1 << (q - 8)) * k8 / 255.0 + 1.0
    T.want, T.tol, T.rel, T.floor, T.keep, T.skip, T.seg0 = want, tol, rel, floor, keep, skip, seg0
    T.kappa, T.U = kappa, U
    return T


def judge_float(params, kernel, kind, stage, got, T):
    """Evaluate got (3, H, W) against a Tolerance; returns (report, failures).
    Pure: no assertion, no I/O."""
    want, tol, rel, floor, keep = T.want, T.tol, T.rel, T.floor, T.keep
    fails = []
    got = got.astype(np.float64)
    with np.errstate(invalid='ignore'):
        err = np.abs(got - want)
    if T.skip.mean() >= (0.1 if kind == 'edges' else 0.01):
        fails.append(f'{T.skip.mean():.2%} of pixels excluded as ill-conditioned')
    if not (np.isfinite(want[keep]).all() and np.isfinite(got[keep]).all()):
        fails.append('non-finite values among the kept pixels')
    with np.errstate(invalid='ignore', divide='ignore'):
        beyond_rel = keep & (err > rel)
        near_zero = keep & (np.abs(want) < 1e-3 * np.broadcast_to(floor, want.shape))
        floor_only = beyond_rel & (err <= tol) & ~near_zero
        relerr = np.where(keep & ~beyond_rel & (np.abs(want) > 0), err / np.abs(want), 0.0)
        # values where a 2e-3 relative error would pass unnoticed (the gate's
        # allowance there exceeds twice the 1e-3 it states), among the values
        # that have a relative scale: above the stage's floor scale and at
        # least 1 % of their pixel's largest channel (a channel the IPT rows or
        # desaturation cancel to ~0 is judged by its absolute uncertainty)
        T.scaled = keep & (np.abs(want) > np.broadcast_to(floor, want.shape) / 1e-3) & \
            (np.abs(want) >= 0.01 * np.nanmax(np.abs(np.nan_to_num(want)), axis=0, keepdims=True))
        loose = T.scaled & (tol > 2e-3 * np.abs(want))
    nk = max(1, int(keep.sum()))
    report = dict(kernel=kernel, cfg=None, kind=kind, stage=stage, values=int(want.size),
                  excluded_px=int(T.skip.sum()), excluded_frac=float(T.skip.mean()),
                  floor_set_frac=float((keep & (np.broadcast_to(floor, want.shape) > rel)).sum() / nk),
                  floor_only_frac=float(floor_only.sum() / nk),
                  near_zero_frac=float((beyond_rel & near_zero).sum() / nk),
                  loose_frac=float(loose.sum() / max(1, int(T.scaled.sum()))),
                  max_rel_err_rest=float(relerr.max(initial=0.0)))
    if T.near_tie is not None:
        # libplacebo branch after the 8-bit download: a pixel may differ only
        # where its download can round the other way (a stage-3 channel within
        # TIE_WINDOW codes of the boundary), by at most the k8 bound, and on
        # fewer than 1 % of the pixels
        flip = ((err > tol) & keep).any(axis=0)
        report['flip_frac'] = float(flip.mean())
        if flip.mean() >= 0.01:
            fails.append(f'{flip.mean():.3%} of pixels off after the rgba8 download')
        if (flip & ~T.near_tie).any():
            fails.append(f'{int((flip & ~T.near_tie).sum())} pixels off with no download channel near its '
                         f'rounding boundary')
        if not (err[keep] <= T.flip_lim).all():
            fails.append(f'max {float(err[keep].max()):.4g} > {T.flip_lim:.4g}')
        return report, fails
    bad = (err > tol) & keep
    if bad.any():
        i = int(np.argmax(np.where(bad, err / tol, 0)))
        fails.append(f'{kernel} stage {stage}: {int(bad.sum())} values beyond 1e-3 rel + {float(np.max(floor)):g} '
                     f'({int(T.skip.sum())} ill-conditioned pixels excluded); worst: want '
                     f'{float(want.flat[i]):.6g} got {float(got.flat[i]):.6g}')
    if report['floor_only_frac'] > FLOOR_ONLY_MAX[kind]:
        fails.append(f'{report["floor_only_frac"]:.2%} of values pass only through the floor '
                     f'(bound {FLOOR_ONLY_MAX[kind]:.0%})')
    return report, fails
