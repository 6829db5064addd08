"""Oracle self-checks on CPU: known answers of each restated stage, the
reference's parameter defaults, and frame-level properties.  The LUT stage
itself is pinned against the reference generator in test_lut.py."""
import math

import numpy as np
import pytest

import oracle
import hdr2sdr
from hdr2sdr.synth import synth_frames

TM = {'none': 0, 'linear': 1, 'gamma': 2, 'clip': 3, 'reinhard': 4, 'hable': 5, 'mobius': 6, 'bt.2390': 7,
      'spline': 8}


def params(**kw):
    if 'tonemap' in kw and isinstance(kw['tonemap'], str):
        kw['tonemap'] = TM[kw['tonemap']]
    return oracle.default_params(**kw)


# ---- S1: ST 2084 / ARIB B67 (zimg) ---------------------------------------
@pytest.mark.parametrize('code,nits', [(0.0, 0.0), (1.0, 10000.0), (0.5080784, 100.0), (0.7518271, 1000.0),
                                       (0.9025723, 4000.0)])
def test_pq_eotf_known_points(code, nits):
    assert oracle.pq_eotf(code) * 10000.0 == pytest.approx(nits, rel=2e-5, abs=1e-6)


def test_pq_eotf_clamps_negative_and_subthreshold():
    assert oracle.pq_eotf(-0.3) == 0.0
    assert oracle.pq_eotf(1e-8) == 0.0          # E^(1/m2) < c1 -> 0


def test_hlg_inverse_oetf_known_points():
    assert oracle.hlg_inverse_oetf(0.5) == pytest.approx(1.0 / 12.0, rel=1e-6)
    assert oracle.hlg_inverse_oetf(0.25) == pytest.approx(0.25 ** 2 / 3.0, rel=1e-6)
    assert oracle.hlg_inverse_oetf(1.0) == pytest.approx(1.0, rel=1e-5)
    assert oracle.hlg_inverse_oetf(-1.0) == 0.0


# ---- S2: vf_tonemap curves and init defaults -------------------------------
def test_tonemap_param_defaults_match_vf_tonemap():
    assert oracle.resolved(params(tonemap='reinhard'))[1] == 1.0          # NaN -> 1.0
    assert oracle.resolved(params(tonemap='reinhard', tm_param=0.5))[1] == 1.0   # (1-p)/p
    assert oracle.resolved(params(tonemap='reinhard', tm_param=0.25))[1] == 3.0
    assert oracle.resolved(params(tonemap='mobius'))[1] == pytest.approx(0.3)
    assert oracle.resolved(params(tonemap='gamma'))[1] == pytest.approx(1.8)
    assert oracle.resolved(params(tonemap='hable'))[1] == 1.0


@pytest.mark.parametrize('kw,peak', [({}, 10.0), ({'maxcll': 1000.0}, 10.0), ({'mastering_max': 4000.0}, 40.0),
                                     ({'maxcll': 400.0, 'mastering_max': 1000.0}, 4.0), ({'peak': 5.0}, 5.0)])
def test_signal_peak_resolution(kw, peak):
    """ff_determine_signal_peak: MaxCLL, then mastering max, then the
    linear-trc default 10 (REFERENCE_WHITE 100)."""
    assert oracle.resolved(params(**kw))[0] == pytest.approx(peak)


def test_tone_curve_known_answers():
    assert oracle.tone_curve(params(tonemap='hable'), 10.0) == pytest.approx(1.0, rel=1e-6)      # sig = peak
    assert oracle.tone_curve(params(tonemap='reinhard'), 10.0) == pytest.approx(1.0, rel=1e-6)
    assert oracle.tone_curve(params(tonemap='mobius'), 0.2) == pytest.approx(0.2, rel=1e-7)      # identity <= j
    assert oracle.tone_curve(params(tonemap='mobius'), 10.0) == pytest.approx(1.0, rel=1e-5)
    assert oracle.tone_curve(params(tonemap='linear'), 2.0) == pytest.approx(0.2, rel=1e-6)      # sig * 1/peak
    assert oracle.tone_curve(params(tonemap='clip'), 3.0) == pytest.approx(1.0)
    assert oracle.tone_curve(params(tonemap='none'), 3.0) == pytest.approx(3.0)
    # hable(0)-based curve passes through ~0 and is monotonic
    xs = np.linspace(1e-4, 20, 200)
    ys = [oracle.tone_curve(params(tonemap='hable'), float(x)) for x in xs]
    assert ys[0] < 1e-3 and all(b >= a for a, b in zip(ys, ys[1:]))


PIPE_CPU, PIPE_LP = 1, 2


@pytest.mark.parametrize('knee', [0.5, 1.0])
def test_bt2390_eetf_shape(knee):
    """CPU-chain target (npl white, no black): identity below the knee, the
    source peak onto the target white, clipped above the source range."""
    p = params(tonemap='bt.2390', pipeline=PIPE_CPU, knee_offset=knee)
    assert oracle.tone_curve(p, 0.01) == pytest.approx(0.01, rel=1e-3)     # below the knee: identity
    top = oracle.tone_curve(p, 10.0)                                        # source peak -> target peak
    assert top == pytest.approx(1.0, rel=1e-3)
    assert oracle.tone_curve(p, 100.0) == pytest.approx(top, rel=1e-6)      # clipped to source range


def _bt2390_ref(sig, peak=10.0, white=203.0, black=0.203, offset=1.0):
    """Independent double transcription of libplacebo's bt2390 (knee offset,
    black-point adaptation); sig in units of 100 nits, output in units of the
    target white."""
    smin, smax = _pq_enc(0.0), _pq_enc(peak / 100.0)
    ml = (_pq_enc(white / 10000.0) - smin) / (smax - smin)
    mn = (_pq_enc(black / 10000.0) - smin) / (smax - smin) if black > 0 else 0.0
    ks = (1 + offset) * ml - offset
    bp = min(1 / mn, 4.0) if mn > 0 else 4.0
    gain = 1 / (1 + mn / ml * (1 - ml) ** bp) if ml < 1 else 1.0
    x = min(max((_pq_enc(sig / 100.0) - smin) / (smax - smin), 0.0), 1.0)
    if ks < 1 and x > ks:
        t = (x - ks) / (1 - ks)
        x = (2 * t ** 3 - 3 * t ** 2 + 1) * ks + (t ** 3 - 2 * t ** 2 + t) * (1 - ks) + (-2 * t ** 3 + 3 * t ** 2) * ml
    if mn > 0 and x < 1:
        x += mn * (1 - x) ** bp
        x = gain * (x - mn) + mn
    return oracle.pq_eotf_d(x * (smax - smin) + smin) * 10000.0 / white


@pytest.mark.parametrize('peak,knee,black', [(10.0, 1.0, None), (40.0, 1.0, None), (10.0, 0.5, None),
                                             (10.0, 1.0, 0.0), (4.0, 2.0, 1.0)])
def test_bt2390_libplacebo_matches_independent_transcription(peak, knee, black):
    """libplacebo branch defaults: 203-nit white, 1000:1 black, knee offset 1."""
    kw = dict(tonemap='bt.2390', pipeline=PIPE_LP, peak=peak, knee_offset=knee)
    if black is not None:
        kw['target_black'] = black
    p = params(**kw)
    for sig in (1e-4, 0.003, 0.05, 0.2, 0.5, 1.0, 2.0, 5.0, peak * 0.7, peak):
        want = _bt2390_ref(sig, peak=peak, offset=knee, black=0.203 if black is None else black)
        assert oracle.tone_curve(p, sig) == pytest.approx(want, rel=5e-4, abs=1e-6), sig


def test_bt2390_black_point_lifts_black():
    p = params(tonemap='bt.2390', pipeline=PIPE_LP)
    # black maps onto the target black (0.203 of 203 nits = 1e-3 of white)
    assert oracle.tone_curve(p, 1e-6) == pytest.approx(1e-3, rel=5e-2)
    off = params(tonemap='bt.2390', pipeline=PIPE_LP, target_black=0.0)
    assert oracle.tone_curve(off, 1e-6) < 1e-6


# ---- libplacebo spline (PARITY UNPINNED: libplacebo absent) ----------------
def _pq_enc(y):
    m1, m2, c1, c2, c3 = 0.1593017578125, 78.84375, 0.8359375, 18.8515625, 18.6875
    ym = max(y, 0.0) ** m1
    return ((c1 + c2 * ym) / (1 + c3 * ym)) ** m2


def _spline_ref(sig, peak=10.0, npl=100.0, contrast=0.5, avg_pq=0.0, black=0.0, white=None):
    """Second, independent transcription of libplacebo's spline (pick_knee +
    single-pivot toe/shoulder, tone_mapping.c defaults) in double; output in
    units of the target white (default npl)."""
    def smoothstep(e0, e1, x):
        t = min(max((x - e0) / (e1 - e0), 0.0), 1.0)
        return t * t * (3 - 2 * t)
    white = npl if white is None else white
    smin, smax = _pq_enc(0.0), _pq_enc(peak / 100.0)
    dmin, dmax = _pq_enc(black / 10000.0), _pq_enc(white / 10000.0)
    sk = avg_pq if avg_pq > 0 else smin + 0.4 * (smax - smin)
    sk = min(max(sk, smin + 0.1 * (smax - smin)), smin + 0.8 * (smax - smin))
    target = (sk - smin) / (smax - smin)
    adapted = dmin + (dmax - dmin) * target
    tuning = 1 - smoothstep(0.8, 0.4, target) * smoothstep(0.1, 0.4, target)
    dk = min(max(sk + (adapted - sk) * (0.4 + 0.6 * tuning), dmin), dmax)
    ratio = min(max(1.5 * (smax / dmax - 1), 0.2), 1.2)
    slope = (oracle.pq_eotf_d(dk) / oracle.pq_eotf_d(sk)) ** ((1 - contrast) * ratio)
    i0, i1, o0, o1 = smin - sk, smax - sk, dmin - dk, dmax - dk
    x = min(max(_pq_enc(sig * npl / 10000.0), smin), smax) - sk
    if x > 0:
        y = ((((slope * i1 - o1) / (2 * i1 ** 3)) * x - 3 * (slope * i1 - o1) / (2 * i1 * i1)) * x + slope) * x
    else:
        y = ((o0 - slope * i0) / (i0 * i0) * x + slope) * x
    e2 = min(max(y + dk, dmin), dmax)
    return oracle.pq_eotf_d(e2) * 10000.0 / white, sk, dk, slope


@pytest.mark.parametrize('peak,contrast', [(10.0, 0.5), (40.0, 0.5), (10.0, 0.0), (10.0, 1.5), (2.0, 0.5)])
@pytest.mark.parametrize('pipe', [PIPE_CPU, PIPE_LP])
def test_spline_matches_independent_transcription(peak, contrast, pipe):
    p = params(tonemap='spline', peak=peak, tm_param=contrast, pipeline=pipe)
    tgt = dict(black=0.203, white=203.0) if pipe == PIPE_LP else {}
    for sig in (1e-4, 0.003, 0.05, 0.2, 0.5, 1.0, 2.0, 5.0, peak * 0.7, peak, peak * 3):
        want = _spline_ref(sig, peak=peak, contrast=contrast, **tgt)[0]
        assert oracle.tone_curve(p, sig) == pytest.approx(want, rel=2e-4, abs=1e-6), sig


def test_spline_shape():
    p = params(tonemap='spline', pipeline=PIPE_CPU)  # peak 10 (1000 nits), contrast 0.5
    xs = np.geomspace(1e-4, 10.0, 300)
    ys = [oracle.tone_curve(p, float(x)) for x in xs]
    assert all(b >= a - 1e-7 for a, b in zip(ys, ys[1:]))               # monotone
    assert ys[-1] == pytest.approx(1.0, rel=1e-4)                        # source peak -> SDR white
    assert oracle.tone_curve(p, 100.0) == pytest.approx(ys[-1], rel=1e-6)  # clipped to the source range
    _, sk, dk, slope = _spline_ref(1.0)
    assert 0.0 < dk < sk and 0.0 < slope < 1.0       # compressive knee on a 1000-nit source
    # contrast 1 -> the slope exponent is 0: unit PQ-domain slope at the knee
    assert _spline_ref(1.0, contrast=1.0)[3] == pytest.approx(1.0)


# ---- S7: vf_eq create_lut ---------------------------------------------------
def eq_reference(gamma, bits):
    n = 1 << bits
    out = []
    for i in range(n):
        v = i / (n - 1)
        if v <= 0.0:
            out.append(0)
            continue
        v = math.pow(v, 1.0 / gamma)
        out.append(n - 1 if v >= 1.0 else int(n * v))
    return np.array(out)


@pytest.mark.parametrize('gamma', [1.0, 2.2, 0.5, 1.3, 3.0, 0.1])
@pytest.mark.parametrize('mode,bits_out', [(0, 10), (1, 10), (1, 12), (0, 8)])
def test_eq_lut(gamma, mode, bits_out):
    q = bits_out if mode == 1 else 8
    eq = oracle.resolved(params(gamma=gamma, mode=mode, bits_out=bits_out))[2]
    assert np.array_equal(eq, eq_reference(gamma, q))
    if gamma == 1.0:
        assert np.array_equal(eq, np.arange(1 << q))


# ---- frame level ----------------------------------------------------------
LAT = None


def lattice():
    global LAT
    if LAT is None:
        LAT = hdr2sdr.generate_lattice(65)
    return LAT


def grey_frames(bits=10, w=64, h=8):
    fb = hdr2sdr.FrameBatch.empty_numpy(1, w, h, bits)
    s = 1 << (bits - 8)
    fb.y[0] = np.linspace(16 * s, 235 * s, w).astype(np.uint16)[None, :]
    fb.u[0] = 128 * s
    fb.v[0] = 128 * s
    return fb


@pytest.mark.parametrize('tm', ['reinhard', 'hable', 'mobius', 'bt.2390'])
@pytest.mark.parametrize('bits', [10, 12])
def test_neutral_axis_stays_neutral_and_monotonic(tm, bits):
    fb = grey_frames(bits)
    p = params(tonemap=tm, bits_in=bits, bits_out=bits, transfer_in=0 if bits == 10 else 1)
    out = hdr2sdr.FrameBatch(oracle.process(p, lattice(), fb.buf, fb.width, fb.height), fb.width, fb.height, bits)
    mid = 128 << (bits - 8)
    assert np.abs(out.u.astype(int) - mid).max() <= 1 << (bits - 8)
    assert np.abs(out.v.astype(int) - mid).max() <= 1 << (bits - 8)
    row = out.y[0, 0].astype(int)
    assert np.all(np.diff(row) >= 0) and row[0] == 16 << (bits - 8)


def test_compat8_output_is_8bit_shifted_and_native_is_not():
    fb = synth_frames('smooth', 1, 64, 32, 10, seed=4).to_numpy()
    c8 = oracle.process(params(tonemap='hable', mode=0), lattice(), fb.buf, 64, 32)
    nat = oracle.process(params(tonemap='hable', mode=1), lattice(), fb.buf, 64, 32)
    assert np.all(c8 % 4 == 0)
    assert np.any(nat % 4 != 0)
    assert np.abs(c8.astype(int) - nat.astype(int)).max() <= 4


def test_lut_chain_tracks_closed_form_gamut_math():
    """Analog of the reference smoke test TestLutReproducesLegacyGamutMath
    (test/smoke_test.py:264-343): the 65^3 tetrahedral LUT chain and the
    closed-form zscale p=bt709 chain (FFMPEG_FILTER_LEGACY_NO_LUT) agree within
    12/255 on a 21x21 sample grid (reference tolerance :300)."""
    W, H = 960, 540
    fb = synth_frames('smooth', 1, W, H, 10, seed=21).to_numpy()
    lut_rgb = oracle.debug_float(params(tonemap='reinhard'), lattice(), fb.buf, W, H, 4)
    legacy = oracle.debug_float(params(tonemap='reinhard', lut_enabled=0), None, fb.buf, W, H, 4)
    ys = np.arange(0, H, max(1, H // 20))
    xs = np.arange(0, W, max(1, W // 20))
    a = np.round(np.clip(lut_rgb[:, ys][:, :, xs], 0, 1) * 255)
    b = np.round(np.clip(legacy[:, ys][:, :, xs], 0, 1) * 255)
    assert np.abs(a - b).max() <= 12


def test_multithreaded_oracle_is_deterministic():
    fb = synth_frames('uniform', 3, 128, 64, 10, seed=2).to_numpy()
    p = params(tonemap='hable', gamma=2.2)
    a = oracle.process(p, lattice(), fb.buf, 128, 64, nthreads=1)
    b = oracle.process(p, lattice(), fb.buf, 128, 64, nthreads=4)
    assert np.array_equal(a, b)


# ---- S1 chroma upsampler edge rule
def _edge_out(edge, W=64, H=32):
    fb = synth_frames('uniform', 1, W, H, 10, seed=12).to_numpy()
    p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, chroma_edge=edge)
    out = oracle.process(oracle.params_from(p.to_c()), lattice(), fb.buf, W, H)
    o = hdr2sdr.FrameBatch(out, W, H, 10)
    return o.y[0].astype(int), o.u[0].astype(int), o.v[0].astype(int)


def _differs_only_at(a, b, rows, cols):
    d = a != b
    d[list(rows), :] = False
    d[:, list(cols)] = False
    return not d.any()


def test_chroma_edge_rules_act_only_on_the_border():
    """The bilinear upsampler reads past the chroma plane only for luma rows 0
    and H-1 (chroma rows -1 / ch) and the last odd luma column (chroma column
    cw; left siting never reads column -1).  ZIMG and REPLICATE differ at the
    top only (mirror vs repeat of row -1); ZIMG and MIRROR at the bottom and
    right only (fold vs mirror of row ch / column cw)."""
    W, H = 64, 32
    z, r, m = _edge_out('zimg'), _edge_out('replicate'), _edge_out('mirror')
    for a, b, rows, cols, crows, ccols in ((z, r, [0], [], [0], []),
                                          (z, m, [H - 1], [W - 1], [H // 2 - 1], [W // 2 - 1])):
        assert _differs_only_at(a[0], b[0], rows, cols)
        assert _differs_only_at(a[1], b[1], crows, ccols) and _differs_only_at(a[2], b[2], crows, ccols)
        assert any((x != y).any() for x, y in zip(a, b))      # and the rule does change those samples


def test_chroma_edge_single_chroma_row_clamps():
    """1 x 1 chroma planes (2 x 2 luma): every rule stays inside the plane."""
    outs = [_edge_out(e, 2, 2) for e in ('zimg', 'replicate', 'mirror')]
    for o in outs[1:]:
        assert all(np.array_equal(x, y) for x, y in zip(outs[0], o))


def test_chroma_edge_rejects_unknown():
    with pytest.raises(ValueError):
        hdr2sdr.TonemapParams(chroma_edge='wrap')


# ---- S3 -> S4 format -----------------
def test_rgb48_lut_input_is_a_small_perturbation_of_the_float_path():
    """16-bit R'G'B' between zscale and lut3d (rounding in, truncation out, both
    at 1/65535) moves the quantised output by at most one step, on a small
    fraction of samples -- but it does move it (the switch is live)."""
    W, H = 128, 64
    fb = synth_frames('smooth', 2, W, H, 10, seed=13).to_numpy()
    base = hdr2sdr.TonemapParams(tonemapper='hable', gamma=1.0, bits_out=10, mode='native')  # no eq: steps stay steps
    outs = [oracle.process(oracle.params_from(p.to_c()), lattice(), fb.buf, W, H).astype(int)
            for p in (base, base.with_(lut_input='rgb48'))]
    d = np.abs(outs[0] - outs[1])
    assert d.max() <= 1 and 0 < (d > 0).mean() < 0.05


def test_rgb48_lut_stage_values_are_16bit():
    W, H = 64, 32
    fb = synth_frames('ramp', 1, W, H, 10, seed=2).to_numpy()
    p = hdr2sdr.TonemapParams(tonemapper='hable', lut_input='rgb48')
    st4 = oracle.debug_float(oracle.params_from(p.to_c()), lattice(), fb.buf, W, H, 4).astype(np.float64)
    q = st4 * 65535.0
    assert np.allclose(q, np.round(q), atol=2e-3) and st4.min() >= 0 and st4.max() <= 1


def test_lut_input_rejects_unknown():
    with pytest.raises(ValueError):
        hdr2sdr.TonemapParams(lut_input='rgb24')


# ---- libplacebo's reinhard / hable / mobius (PL_HDR_NORM, PARITY UNPINNED) --
def _hable_ref(x):
    a, b, c, d, e, f = 0.15, 0.50, 0.10, 0.20, 0.02, 0.30
    return (x * (x * a + b * c) + d * e) / (x * (x * a + b) + d * f) - e / f


@pytest.mark.parametrize('tm', ['reinhard', 'hable', 'mobius'])
@pytest.mark.parametrize('peak', [10.0, 40.0])
def test_libplacebo_norm_curves_match_independent_transcription(tm, peak):
    """In NORM units (1 = the 203-nit SDR white) the source peak lands on the
    white; reinhard with contrast 0.5, hable over hable(peak), mobius with knee
    0.3 (identity below it); inputs above the source peak clip to it."""
    p = params(tonemap=tm, pipeline=PIPE_LP, peak=peak)
    pk = peak * 100.0 / 203.0
    for sig in (0.01, 0.1, 0.5, 1.0, 2.0, 5.0, peak, 2 * peak):    # units of npl (100 nits)
        x = min(sig * 100.0 / 203.0, pk)
        if tm == 'reinhard':
            off = 1.0
            want = (pk + off) / pk * x / (x + off)
        elif tm == 'hable':
            want = _hable_ref(x) / _hable_ref(pk)
        else:
            j = 0.3
            a = -j * j * (pk - 1) / (j * j - 2 * j + pk)
            b = (j * j - 2 * j * pk + pk) / max(1e-6, pk - 1)
            want = x if x <= j else (b * b + 2 * b * j + j * j) / (b - a) * (x + a) / (x + b)
        assert oracle.tone_curve(p, sig) == pytest.approx(want, rel=2e-5, abs=1e-7), (tm, sig)
    assert oracle.tone_curve(p, peak) == pytest.approx(1.0, rel=1e-5)
