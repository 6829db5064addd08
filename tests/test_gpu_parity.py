"""GPU parity: libh2s (HIP, through the C-ABI) vs the CPU oracle on the same
seeded inputs.

Tolerances (north_star: +-1 LSB after quantisation, 1e-3 relative on the
float path):
* integer output: |gpu - oracle| <= one quantisation step, where the step is
  1 LSB of the depth the chain quantises at — 8 bits in compat8 mode (the
  reference's own precision: eq forces yuv420p, so a 10-bit output moves in
  steps of 4), bits_out in native mode — and fewer than 0.5 % of samples may
  sit one step off (float rounding next to a rounding boundary);
* float intermediates (h2s_debug_float): |gpu - oracle| <= 1e-3 * |oracle| +
  1e-5 absolute floor, per stage.
"""
import ctypes
import math

import numpy as np
import pytest

import oracle
import hdr2sdr
from hdr2sdr.synth import synth_frames

pytestmark = pytest.mark.gpu

from float_gate import (EPS_IPT, FLOAT_CFGS, FLOOR_ONLY_MAX, TILE_DARK_EXACT, Planes,  # noqa: F401,E402
                        float_tolerance, judge_float, lattice, lattice_slope, tone_uncertainty)
from float_gate import lattice_max_step as _lattice_max_step  # noqa: E402


@pytest.fixture(scope='module')
def tm():
    t = hdr2sdr.Tonemapper(0)
    yield t
    t.close()


def run_both(tm, params, kind, W, H, nframes=2, lut_n=65, seed=11):
    import torch
    src_cpu = synth_frames(kind, nframes, W, H, params.bits_in, device='cpu', seed=seed)
    src = src_cpu.to_torch('cuda')
    tm.set_params(params)
    if params.lut_enabled:
        tm.set_lut(lattice(lut_n))
    dst = hdr2sdr.FrameBatch.empty_torch(nframes, W, H, params.bits_out, 'cuda')
    tm.process(src, dst)
    torch.cuda.synchronize()
    got = dst.to_numpy().buf.astype(np.int64)
    want = oracle.process(oracle.params_from(params.to_c()), lattice(lut_n) if params.lut_enabled else None,
                          src_cpu.to_numpy().buf, W, H).astype(np.int64)
    return got, want, (W, H, src_cpu.to_numpy().buf)


def parity_report(params, got, want, W, H, q, luma_within=None, attribution=None):
    """Append one JSON line to $H2S_PARITY_REPORT (when set) with the shares
    of output samples that agree exactly with the oracle, sit one quantiser
    step off, and sit further off (a drift inside the
    +-1 step / 0.5 % budget must be visible).  Luma with eq: 'one step'
    means within eq[q-1] .. eq[q+1] of the oracle's code; everything else is
    counted in output steps of the quantiser depth."""
    import json
    import os
    path = os.environ.get('H2S_PARITY_REPORT')
    if not path:
        return None
    step = 1 << max(0, params.bits_out - q)
    ysz = W * H
    d = np.abs(got - want)
    dy, dc = d[:, :ysz], d[:, ysz:]
    y_exact = float((dy == 0).mean())
    y_one = float(luma_within.mean()) - y_exact if luma_within is not None else float(((dy > 0) & (dy <= step)).mean())
    c_exact = float((dc == 0).mean())
    c_one = float(((dc > 0) & (dc <= step)).mean())
    clip = lambda v: max(0.0, v)   # noqa: E731  (float rounding of 1 - a - b)
    rec = dict(test=os.environ.get('PYTEST_CURRENT_TEST', '?').split(' ')[0], pipeline=params.resolved_pipeline(),
               tonemapper=params.tonemapper, bits_in=params.bits_in, bits_out=params.bits_out, gamma=params.gamma,
               W=W, H=H, frames=int(got.shape[0]), quantiser_bits=q,
               luma=dict(exact=y_exact, one_step=y_one, beyond=clip(1.0 - y_exact - y_one)),
               chroma=dict(exact=c_exact, one_step=c_one, beyond=clip(1.0 - c_exact - c_one)),
               # output codes (luma after eq, where one pre-eq step can span several)
               max_diff_out_steps=int(-(-int(d.max(initial=0)) // step)))
    if attribution is not None:   # the libplacebo branch's per-sample tie attribution (tests/lp_gate.py)
        rec['attribution'] = {k: attribution[k] for k in ('beyond', 'attributed', 'unattributed', 'near_tie_px')}
        rec['attribution']['kernel'] = attribution.get('kernel')
    with open(path, 'a') as fh:
        fh.write(json.dumps(rec) + '\n')
    return rec


def assert_close_int(params, got, want, W, H, src=None, max_frac=5e-3, lut_n=65, kernel='k_tile', knees=None):
    """Chroma: |diff| <= one quantisation step.  Luma: eq runs after the
    quantiser, so the bound is +-1 step *before* eq: got must lie between
    eq[q-1] and eq[q+1] where eq[q] == want (eq is monotonic).

    The libplacebo branch with the LUT quantises twice before the output (the
    8-bit rgba download and lut3d's truncating 8-bit output), so a download
    code that rounds the other way moves the output by up to k8 lattice
    steps.  Its gate is tests/lp_gate.py: every sample
    beyond one step must be attributed to a download channel whose exact
    value (oracle.lp_download) lies within `kernel`'s stated stage-3 bound of
    a rounding tie -- 'k_tile' (the default: a superset of the generic
    kernel's), 'exact' (H2S_OPT_LP_EXACT or the generic kernel alone: double
    arithmetic, so in effect none) -- and none may be unattributed.  src: the
    input frames (host numpy) the attribution recomputes; knees: per-frame
    (peak, average) under dynamic peak detection."""
    op = oracle.params_from(params.to_c())
    q = oracle.quant_bits(op)
    if params.resolved_pipeline() == 'libplacebo' and params.lut_enabled:
        import lp_gate
        if src is None:
            raise TypeError('assert_close_int: the libplacebo branch\'s gate needs the input frames (src)')
        rep, fails = lp_gate.check(params, kernel, got, want, src, W, H, lut_n, knees=knees)
        rep['kernel'] = kernel
        parity_report(params, got, want, W, H, q, attribution=rep)
        assert not fails, '; '.join(fails)
        # the share that differs at all (one step, or attributed): twice the
        # CPU chain's budget (round 5's largest: 0.48 %, spline max-rgb HLG12)
        frac = float((np.abs(got - want) > 0).mean())
        budget = 2 * max_frac * (1 << max(0, q - 10))
        assert frac <= budget, f'{frac:.3%} of samples differ (budget {budget:.2%})'
        return
    shift = params.bits_out - q if params.bits_out >= q else 0
    step = 1 << shift
    ysz = W * H
    gy, wy = got[:, :ysz] >> shift, want[:, :ysz] >> shift
    gc, wc = got[:, ysz:], want[:, ysz:]
    if params.expand == 'shift':
        assert np.all(got % step == 0) and np.all(want % step == 0)
    # compared as quantiser codes: a bit-replicated code differs from its
    # neighbour's by step + 1 at the output depth
    dc = np.abs((gc >> shift) - (wc >> shift))
    assert dc.max(initial=0) <= 1, f'chroma max diff {dc.max()} quantiser steps'
    eq = oracle.resolved(op)[2].astype(np.int64)
    lo_i = np.searchsorted(eq, wy, side='left')            # first q with eq[q] == want
    hi_i = np.searchsorted(eq, wy, side='right') - 1       # last q with eq[q] == want
    assert np.all(eq[np.clip(lo_i, 0, len(eq) - 1)] == wy), 'oracle luma not in eq table'
    lo = eq[np.clip(lo_i - 1, 0, len(eq) - 1)]
    hi = eq[np.clip(hi_i + 1, 0, len(eq) - 1)]
    bad = (gy < lo) | (gy > hi)
    parity_report(params, got, want, W, H, q, luma_within=~bad)
    assert not bad.any(), f'{int(bad.sum())} luma samples beyond +-1 pre-eq step'
    # the fraction budget is for quantisers of <= 10 bits; a native 12-bit
    # LSB is 4x finer, so the same float-level disagreement flips 4x as often
    frac = float(((np.abs(got - want)) > 0).mean())
    budget = max_frac * (1 << max(0, q - 10))
    assert frac <= budget, f'{frac:.3%} of samples differ (budget {budget:.2%})'


CONFIGS = {
    # BASELINE.json configs (shrunk to parity sizes)
    'C1_reinhard_33': (dict(tonemapper='reinhard', gamma=1.0, bits_out=10), 33),
    'C2_hable_65_g22': (dict(tonemapper='hable', gamma=2.2, bits_out=10), 65),
    'C3_bt2390': (dict(tonemapper='bt.2390', gamma=1.0, bits_out=10), 65),
    'spline_65': (dict(tonemapper='spline', gamma=1.0, bits_out=10), 65),
    'spline_hlg12_contrast1': (dict(tonemapper='spline', tm_param=1.0, bits_in=12, bits_out=12,
                                    transfer='arib-std-b67'), 65),
    'C4_mobius': (dict(tonemapper='mobius', gamma=1.0, bits_out=10), 65),
    'C5_hlg12_hable': (dict(tonemapper='hable', gamma=1.0, bits_in=12, bits_out=12, transfer='arib-std-b67'), 65),
    'pq12_reinhard_12': (dict(tonemapper='reinhard', gamma=1.0, bits_in=12, bits_out=12), 65),
    'pq12_bt2390_10': (dict(tonemapper='bt.2390', gamma=1.0, bits_in=12, bits_out=10), 65),
    'default_8bit': (dict(tonemapper='mobius', gamma=1.0, bits_out=8), 65),
    'gamma05_8bit': (dict(tonemapper='hable', gamma=0.5, bits_out=8), 65),
}


@pytest.mark.parametrize('kind', ['smooth', 'uniform', 'ramp', 'edges'])
@pytest.mark.parametrize('cfg', sorted(CONFIGS))
def test_configs_match_oracle(tm, cfg, kind):
    kw, lut_n = CONFIGS[cfg]
    params = hdr2sdr.TonemapParams(**kw)
    got, want, src_wh = run_both(tm, params, kind, 128, 64, lut_n=lut_n)
    assert_close_int(params, got, want, *src_wh)


@pytest.mark.parametrize('mode', ['compat8', 'native'])
@pytest.mark.parametrize('tmname', ['none', 'linear', 'gamma', 'clip', 'reinhard', 'hable', 'mobius', 'bt.2390',
                                    'spline'])
def test_every_operator_both_modes(tm, tmname, mode):
    params = hdr2sdr.TonemapParams(tonemapper=tmname, gamma=1.3, bits_out=10, mode=mode)
    got, want, src_wh = run_both(tm, params, 'smooth', 96, 48)
    assert_close_int(params, got, want, *src_wh)


@pytest.mark.parametrize('desat_luma', ['rgb', 'bt2020', 'bt709'])
@pytest.mark.parametrize('desat', [0.0, 2.0, 0.5])
def test_desat_switches(tm, desat_luma, desat):
    params = hdr2sdr.TonemapParams(tonemapper='hable', desat=desat, desat_luma=desat_luma)
    got, want, src_wh = run_both(tm, params, 'uniform', 64, 32)
    assert_close_int(params, got, want, *src_wh)


@pytest.mark.parametrize('peak,maxcll,mastering', [(0, 0, 0), (0, 1000, 0), (0, 0, 4000), (0, 400, 1000), (5.0, 0, 0)])
def test_peak_sources(tm, peak, maxcll, mastering):
    params = hdr2sdr.TonemapParams(tonemapper='reinhard', peak=peak, maxcll=maxcll, mastering_max=mastering)
    got, want, src_wh = run_both(tm, params, 'ramp', 64, 32)
    assert_close_int(params, got, want, *src_wh)


@pytest.mark.parametrize('W,H', [(2, 2), (4, 2), (6, 4), (18, 6), (130, 10), (1922, 4)])
def test_ragged_sizes_scalar_path(tm, W, H):
    """Widths that are not a multiple of the 8-pixel vector group, and
    1-row / 1-column chroma planes (edge rules on both sides)."""
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
    got, want, src_wh = run_both(tm, params, 'uniform', W, H, nframes=3)
    assert_close_int(params, got, want, *src_wh)


@pytest.mark.parametrize('bits_in,transfer', [(10, 'smpte2084'), (12, 'arib-std-b67')])
@pytest.mark.parametrize('bits_out', [10, 8])
@pytest.mark.parametrize('W,H', [(80, 34), (352, 64), (720, 48), (1440, 36)])
def test_tile_plus_tail_widths(tm, W, H, bits_out, bits_in, transfer):
    """Widths that are not a multiple of 64 with 16-byte aligned rows: whole
    64-pixel tiles go through k_tile and the remaining columns through
    k_process from the same chroma group on (the seam sits at W & ~63)."""
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_in=bits_in, bits_out=bits_out,
                                   transfer=transfer)
    for kind in ('uniform', 'smooth'):
        got, want, src_wh = run_both(tm, params, kind, W, H, nframes=2)
        assert_close_int(params, got, want, *src_wh)


def test_lut_disabled_closed_form(tm):
    params = hdr2sdr.TonemapParams(tonemapper='hable', lut_enabled=False)
    got, want, src_wh = run_both(tm, params, 'ramp', 128, 64)
    assert_close_int(params, got, want, *src_wh)


@pytest.mark.parametrize('lut_n', [2, 17, 33, 65, 129, 177, 178, 200, 256])
def test_lut_sizes(tm, lut_n):
    """Every lut3d size (MAX_LEVEL 256).  The tile kernel forms lattice byte
    offsets in float32 (exact below 2^26 for multiples of 4, i.e. N <= 177);
    larger lattices take the generic kernel (h2s_query_path)."""
    from hdr2sdr import _abi
    params = hdr2sdr.TonemapParams(tonemapper='mobius')
    got, want, src_wh = run_both(tm, params, 'uniform', 64, 32, lut_n=lut_n)
    assert_close_int(params, got, want, *src_wh)
    src = hdr2sdr.FrameBatch.empty_torch(1, 64, 32, 10, 'cuda')
    dst = hdr2sdr.FrameBatch.empty_torch(1, 64, 32, 10, 'cuda')
    assert tm.query_path(src, dst) == (_abi.PATH_TILE if lut_n <= 177 else _abi.PATH_GENERIC)


@pytest.mark.parametrize('lut_n', [2, 17, 33, 129, 177, 200, 256])
def test_lut_sizes_libplacebo(tm, lut_n):
    """lut3d's 8-bit path on the libplacebo branch at other lattice sizes:
    k_tile<..., LP=1> reads lut3d's output for its three rgba codes from the
    context's 2^24-entry table (k_build_lut8x: (q / 255) (N-1), N - 1 a
    power of two or not, the code 255 on the last node), so every N up to
    256 stays on the tile path."""
    from hdr2sdr import _abi
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', pipeline='libplacebo')
    got, want, src_wh = run_both(tm, params, 'uniform', 64, 32, lut_n=lut_n)
    assert_close_int(params, got, want, *src_wh, lut_n=lut_n)
    src = hdr2sdr.FrameBatch.empty_torch(1, 64, 32, 10, 'cuda')
    dst = hdr2sdr.FrameBatch.empty_torch(1, 64, 32, 10, 'cuda')
    assert tm.query_path(src, dst) == _abi.PATH_TILE


def _morton_to_linear():
    """For each index of the tile kernel's bit-interleaved table, the linear
    index r | g << 8 | b << 16 of its code triple."""
    i = np.arange(1 << 24, dtype=np.uint32)
    r = np.zeros_like(i)
    g = np.zeros_like(i)
    b = np.zeros_like(i)
    for k in range(8):
        r |= ((i >> (3 * k)) & 1) << k
        g |= ((i >> (3 * k + 1)) & 1) << k
        b |= ((i >> (3 * k + 2)) & 1) << k
    return r | (g << 8) | (b << 16)


@pytest.mark.parametrize('lut_n', [2, 33, 65, 177, 256])
def test_lut8x_table_equals_the_oracle_lut3d_8bit(lut_n):
    """The libplacebo branch's lut3d table (k_build_lut8x, through the
    private entry h2stest_lut8x) equals the oracle's lut3d 8-bit path for
    every one of the 2^24 rgba8 code triples, bit for bit."""
    from hdr2sdr import _abi
    L = ctypes.CDLL(_abi.LIB_PATH)
    L.h2stest_lut8x.restype = ctypes.c_int
    L.h2stest_lut8x.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lat = np.ascontiguousarray(lattice(lut_n), dtype=np.float32)
    got = np.empty(1 << 24, dtype=np.uint32)
    assert L.h2stest_lut8x(lat.ctypes.data, lut_n, got.ctypes.data) == 0
    want = oracle.lut8x_table(lat)[_morton_to_linear()]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad.size, [(int(i), hex(int(got[i])), hex(int(want[i]))) for i in bad[:5]])


def test_lut8x_table_rebuilt_after_set_lut(tm):
    """The 8-bit table follows the lattice: a new h2s_set_lut (another size,
    then the first again) changes the branch's output as the oracle's."""
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', pipeline='libplacebo')
    for n in (33, 65, 33):
        got, want, src_wh = run_both(tm, params, 'smooth', 128, 64, lut_n=n)
        assert_close_int(params, got, want, *src_wh, lut_n=n)


# 1e-3 relative on the float path (north_star), per stage, on the kernel that
# produces the output: k_tile's own debug instance (H2S_OPT_FAST_PATH 1, the
# tile path) and the generic kernel (FAST_PATH 0).  The gate itself (what is
# allowed beyond 1e-3 and why) is tests/float_gate.py, shared with the CPU
# mutation tests of tests/test_float_gate.py that show it rejects real errors.
def check_float_stage(tm, kernel, cfg, kind, stage, W=128, H=64):
    """One (kernel, config, content, stage) float check; returns its report."""
    import json
    import os
    from hdr2sdr import _abi
    params = hdr2sdr.TonemapParams(**FLOAT_CFGS[cfg])
    src = synth_frames(kind, 1, W, H, params.bits_in, device='cpu', seed=3)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    tm.set_option(_abi.OPT_FAST_PATH, 1 if kernel == 'k_tile' else 0)
    try:
        dsrc = src.to_torch('cuda')
        path = tm.query_path(dsrc, hdr2sdr.FrameBatch.empty_torch(1, W, H, params.bits_out, 'cuda'))
        assert path == (_abi.PATH_TILE if kernel == 'k_tile' else _abi.PATH_GENERIC)
        got = tm.debug_float(dsrc, stage)
    finally:
        tm.set_option(_abi.OPT_FAST_PATH, 1)
    T = float_tolerance(params, kernel, stage, kind, Planes(params, src.to_numpy().buf, W, H))
    report, fails = judge_float(params, kernel, kind, stage, got, T)
    report['cfg'] = cfg
    if os.environ.get('H2S_FLOAT_REPORT'):
        with open(os.environ['H2S_FLOAT_REPORT'], 'a') as fh:
            fh.write(json.dumps(report) + '\n')
    if os.environ.get('H2S_FLOOR_ONLY_MAX'):        # (a survey run may lift the floor-only bound)
        bound = float(os.environ['H2S_FLOOR_ONLY_MAX'])
        fails = [f for f in fails if 'pass only through the floor' not in f or report['floor_only_frac'] > bound]
    if os.environ.get('H2S_FLOAT_DEBUG') and fails:   # the worst few, with what their tolerance was made of
        err = np.abs(got.astype(np.float64) - T.want)
        bad = (err > T.tol) & T.keep
        for i in np.argsort(np.where(bad, err / T.tol, 0).ravel())[::-1][:4]:
            c, y, x = np.unravel_index(i, T.want.shape)
            print(f'  [{kernel} {cfg} {kind} s{stage}] c{c} ({y},{x}) want {T.want[c, y, x]:.6g} '
                  f'got {got[c, y, x]:.6g} tol {T.tol[c, y, x]:.3g} kappa {T.kappa[y, x]:.3g}', flush=True)
    assert not fails, '; '.join(fails)
    return report


@pytest.mark.parametrize('stage', [1, 2, 3, 4, 5])
@pytest.mark.parametrize('kind', ['uniform', 'edges', 'ramp'])
@pytest.mark.parametrize('cfg', sorted(FLOAT_CFGS))
@pytest.mark.parametrize('kernel', ['k_tile', 'k_debug'])
def test_float_intermediates_within_1e3(tm, kernel, cfg, kind, stage):
    check_float_stage(tm, kernel, cfg, kind, stage)


def test_host_memory_path_equals_device_path(tm):
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    src = synth_frames('smooth', 3, 256, 64, 10, device='cpu', seed=5)
    host_out = tm(src.to_numpy())                         # PCIe-inclusive path
    dev_out = tm(src.to_torch('cuda')).to_numpy()
    assert np.array_equal(host_out.buf, dev_out.buf)


@pytest.mark.parametrize('where', ['host_host', 'host_dev', 'dev_host'])
def test_pipelined_host_path_equals_device_path(tm, where):
    """h2s_process cuts a host batch into chunks (H2D | kernel | D2H on three
    streams): 11 frames -> 6 uneven chunks, each side host or device."""
    import torch
    params = hdr2sdr.TonemapParams(tonemapper='reinhard', gamma=1.4)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    F, W, H = 11, 512, 128
    src = synth_frames('uniform', F, W, H, 10, device='cpu', seed=21)
    want = tm(src.to_torch('cuda')).to_numpy().buf
    src_in = src.to_numpy() if where.startswith('host') else src.to_torch('cuda')
    dst = (hdr2sdr.FrameBatch.empty_pinned(F, W, H, 10) if where.endswith('host')
           else hdr2sdr.FrameBatch.empty_torch(F, W, H, 10, 'cuda'))
    tm.process(src_in, dst)
    torch.cuda.synchronize()
    assert np.array_equal(dst.to_numpy().buf, want)


def test_pipelined_host_path_padded_host_layout(tm):
    """Host frames with row padding and frame gaps (per-plane 2D copies per
    chunk) through the pipeline equal the tight device result."""
    import ctypes
    import torch
    W, H, F, bits_out = 256, 64, 5, 10
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=bits_out)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    src = synth_frames('smooth', F, W, H, 10, device='cpu', seed=3)
    want = tm(src.to_torch('cuda')).to_numpy().buf
    probe = torch.zeros(1, dtype=torch.uint8)
    _, in_ls, in_fp = _padded_descriptor(probe, W, H, 10, 32, 4096)
    raw_in = torch.from_numpy(_pack_padded(src.to_numpy().buf, W, H, 10, in_ls, in_fp)).pin_memory()
    in_d, _, _ = _padded_descriptor(raw_in, W, H, 10, 32, 4096)
    _, out_ls, out_fp = _padded_descriptor(probe, W, H, bits_out, 64, 512)
    raw_out = torch.zeros(F * out_fp + 64, dtype=torch.uint8).pin_memory()
    out_d, _, _ = _padded_descriptor(raw_out, W, H, bits_out, 64, 512)
    from hdr2sdr import _abi
    in_d.location = out_d.location = _abi.LOC_HOST
    tm._check(tm._L.h2s_process(tm._ctx, ctypes.byref(in_d), ctypes.byref(out_d), F, None))
    got = _unpack_padded(raw_out.numpy(), F, W, H, bits_out, out_ls, out_fp)
    assert np.array_equal(got.reshape(F, -1), want.reshape(F, -1))


def test_serial_host_schedule_equals_pipelined(tm, monkeypatch):
    params = hdr2sdr.TonemapParams(tonemapper='mobius', gamma=1.0)
    src = synth_frames('smooth', 7, 256, 64, 10, device='cpu', seed=8).to_numpy()
    tm.set_params(params)
    tm.set_lut(lattice(65))
    piped = tm(src).buf
    monkeypatch.setenv('H2S_HOST_SERIAL', '1')
    ser = hdr2sdr.Tonemapper(0, params, lattice(65))
    try:
        assert np.array_equal(ser(src).buf, piped)
    finally:
        ser.close()


def test_batch_equals_single_frames(tm):
    import torch
    params = hdr2sdr.TonemapParams(tonemapper='mobius', gamma=0.8)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    src = synth_frames('uniform', 4, 256, 128, 10, device='cpu', seed=9).to_torch('cuda')
    whole = tm(src).to_numpy().buf
    for i in range(4):
        one = tm(src.slice(i, i + 1)).to_numpy().buf
        assert np.array_equal(one[0], whole[i])
    torch.cuda.synchronize()


def test_errors_map_to_reference_exceptions(tm):
    params = hdr2sdr.TonemapParams(tonemapper='hable')
    tm.set_params(params)
    tm.set_lut(lattice(65))      # so the bits mismatch, not LUT_MISSING, is hit
    src = synth_frames('uniform', 1, 64, 32, 10, device='cpu').to_torch('cuda')
    bad = hdr2sdr.FrameBatch.empty_torch(1, 64, 32, 8, 'cuda')   # bits mismatch
    with pytest.raises(ValueError):
        tm.process(src, bad)
    fresh = hdr2sdr.Tonemapper(0, params)                  # no LUT loaded
    with pytest.raises(FileNotFoundError):
        fresh(src)
    fresh.close()


def test_empty_and_negative_batches(tm):
    """nframes=0 is a no-op that leaves dst untouched (an empty pipe read in
    the planner); nframes<0 is INVALID_ARG -> ValueError, like every other
    impossible request (src/ffmpeg_command.py:240-245)."""
    import torch
    tm.set_params(hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=10))
    tm.set_lut(lattice(65))
    src = synth_frames('smooth', 2, 128, 64, 10, device='cpu').to_torch('cuda')
    dst = hdr2sdr.FrameBatch.empty_torch(2, 128, 64, 10, 'cuda')
    dst.buf.fill_(0x1234)
    tm.process(src, dst, nframes=0)
    torch.cuda.synchronize()
    assert bool((dst.buf == 0x1234).all())
    with pytest.raises(ValueError):
        tm.process(src, dst, nframes=-1)
    with pytest.raises(ValueError):
        tm.process(src, dst, nframes=3)          # more than the batch holds
    tm.process(src, dst, nframes=1)              # only frame 0 is written
    torch.cuda.synchronize()
    assert not bool((dst.buf[0] == 0x1234).all())
    assert bool((dst.buf[1] == 0x1234).all())


def _padded_descriptor(buf, W, H, bits, ls_pad, fp_pad):
    """h2s_frames over a torch uint8 byte buffer with row padding and frame gaps."""
    from hdr2sdr import _abi
    sb = 1 if bits == 8 else 2
    ls = [W * sb + ls_pad, W // 2 * sb + ls_pad // 2, W // 2 * sb + ls_pad // 2]
    ysz, csz = H * ls[0], H // 2 * ls[1]
    fp = ysz + 2 * csz + fp_pad
    d = _abi.H2SFrames()
    base = buf.data_ptr()
    d.data[0], d.data[1], d.data[2] = base, base + ysz, base + ysz + csz
    for p in range(3):
        d.linesize[p], d.frame_pitch[p] = ls[p], fp
    d.width, d.height, d.bits, d.location = W, H, bits, _abi.LOC_DEVICE
    return d, ls, fp


def _pack_padded(tight, W, H, bits, ls, fp):
    """Copy a tight [F, W*H*3/2] batch into a padded byte layout (numpy)."""
    sb = 1 if bits == 8 else 2
    F = tight.shape[0]
    raw = np.zeros((F * fp + 64,), dtype=np.uint8)
    tb = tight.view(np.uint8).reshape(F, -1)
    for f in range(F):
        off_t, off_p = 0, f * fp
        for p, (w, h) in enumerate(((W, H), (W // 2, H // 2), (W // 2, H // 2))):
            for r in range(h):
                raw[off_p + r * ls[p]: off_p + r * ls[p] + w * sb] = tb[f, off_t + r * w * sb: off_t + (r + 1) * w * sb]
            off_t += w * h * sb
            off_p += h * ls[p]
    return raw


def _unpack_padded(raw, F, W, H, bits, ls, fp):
    sb = 1 if bits == 8 else 2
    out = np.zeros((F, W * H * 3 // 2 * sb), dtype=np.uint8)
    for f in range(F):
        off_t, off_p = 0, f * fp
        for p, (w, h) in enumerate(((W, H), (W // 2, H // 2), (W // 2, H // 2))):
            for r in range(h):
                out[f, off_t + r * w * sb: off_t + (r + 1) * w * sb] = raw[off_p + r * ls[p]: off_p + r * ls[p] + w * sb]
            off_t += w * h * sb
            off_p += h * ls[p]
    return out.view(np.uint8 if bits == 8 else np.uint16)


@pytest.mark.parametrize('bits_out', [10, 8])
def test_padded_strides_and_frame_gaps(tm, bits_out):
    """Row padding (linesize > width) and gaps between frames, on both sides,
    through the tile kernel (16-byte aligned) — equal to the tight result."""
    import ctypes
    import torch
    W, H, F = 256, 96, 3
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=bits_out)
    got_tight, want, _ = run_both(tm, params, 'smooth', W, H, nframes=F)
    src = synth_frames('smooth', F, W, H, 10, device='cpu', seed=11).to_numpy()
    # input: 32 bytes of row padding, 4 KiB between frames
    probe = torch.zeros(1, dtype=torch.uint8)
    _, in_ls, in_fp = _padded_descriptor(probe, W, H, 10, 32, 4096)
    raw_in = torch.from_numpy(_pack_padded(src.buf, W, H, 10, in_ls, in_fp)).cuda()
    in_d, _, _ = _padded_descriptor(raw_in, W, H, 10, 32, 4096)
    _, out_ls, out_fp = _padded_descriptor(probe, W, H, bits_out, 64, 512)
    raw_out = torch.zeros(F * out_fp + 64, dtype=torch.uint8, device='cuda')
    out_d, _, _ = _padded_descriptor(raw_out, W, H, bits_out, 64, 512)
    tm._check(tm._L.h2s_process(tm._ctx, ctypes.byref(in_d), ctypes.byref(out_d), F, None))
    torch.cuda.synchronize()
    got = _unpack_padded(raw_out.cpu().numpy(), F, W, H, bits_out, out_ls, out_fp).astype(np.int64)
    assert np.array_equal(got, got_tight)
    assert_close_int(params, got, want, W, H, src.buf)


def test_concurrent_contexts_on_threads_match_serial():
    """The ABI contract (include/h2s.h): any thread may call
    libh2s, one context per worker, no global mutable state.  Four threads,
    each with its own context and operator, process host batches at the same
    time (the ctypes calls release the GIL); every result equals the same
    context's serial result."""
    import threading
    W, H = 256, 128
    cfgs = [dict(tonemapper='hable', gamma=2.2), dict(tonemapper='mobius'), dict(tonemapper='spline'),
            dict(tonemapper='bt.2390', bits_out=8)]
    srcs = [synth_frames(k, 3, W, H, 10, device='cpu', seed=50 + i).to_numpy()
            for i, k in enumerate(('smooth', 'uniform', 'ramp', 'edges'))]
    ctxs = [hdr2sdr.Tonemapper(0, hdr2sdr.TonemapParams(**c), lattice(65)) for c in cfgs]
    outs = [[None] * 5 for _ in ctxs]
    errs = []

    def work(i):
        try:
            for r in range(5):
                dst = hdr2sdr.FrameBatch.empty_numpy(3, W, H, ctxs[i].params.bits_out)
                ctxs[i].process(srcs[i], dst)
                outs[i][r] = dst.buf.copy()
        except Exception as e:  # surfaced below
            errs.append(e)
    threads = [threading.Thread(target=work, args=(i,)) for i in range(len(ctxs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=60)
    assert not errs, errs
    for i, c in enumerate(ctxs):
        dst = hdr2sdr.FrameBatch.empty_numpy(3, W, H, c.params.bits_out)
        c.process(srcs[i], dst)
        for r in range(5):
            assert np.array_equal(outs[i][r], dst.buf), (cfgs[i], r)
        c.close()


def test_set_params_waits_only_for_its_own_context():
    """h2s_set_params / h2s_set_lut drain the context's OWN queued launches
    (events recorded after them), not the device: with
    a ~0.3 s spin kernel queued on a side stream, ahead of context A's launch
    on that stream, context B's set_params returns at once, while A's waits
    for its launch (and so for the spin ahead of it)."""
    import time
    import torch
    W, H = 256, 128
    p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
    a = hdr2sdr.Tonemapper(0, p, lattice(65))
    b = hdr2sdr.Tonemapper(0, p, lattice(65))
    src = synth_frames('smooth', 2, W, H, 10, device='cpu', seed=4).to_torch('cuda')
    dst = hdr2sdr.FrameBatch.empty_torch(2, W, H, 10, 'cuda')
    b.process(src, dst)          # b has launched before (its own events drain at once)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    # calibrate torch's spin kernel (its cycle counter's rate) to ~0.3 s
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(50_000_000)
    torch.cuda.synchronize()
    spin = int(50_000_000 * 0.3 / max(time.perf_counter() - t0, 1e-4))
    try:
        with torch.cuda.stream(side):
            torch.cuda._sleep(spin)
        a.process(src, dst, side)                       # queued behind the spin
        t0 = time.perf_counter()
        b.set_params(p.with_(gamma=1.5))
        b.set_lut(lattice(33))
        tb = time.perf_counter() - t0
        t0 = time.perf_counter()
        a.set_params(p.with_(gamma=1.5))
        ta = time.perf_counter() - t0
        torch.cuda.synchronize()
        assert tb < 0.1, f'set_params on B waited {tb:.3f} s for work that is not its own'
        assert ta > 0.1, f'set_params on A returned after {ta:.3f} s, before its queued launch ran'
    finally:
        a.close()
        b.close()


def test_set_params_waits_for_a_failed_calls_queued_launch():
    """an h2s_process that fails after queueing its kernels (here
    the H2S_OPT_TEST_FAIL_AFTER_LAUNCH test hook, standing in for a D2H copy or
    event failure) still records its launch, so the same context's next
    set_params waits for the queued kernel (queued behind a ~0.3 s spin)
    before rewriting the tables it reads."""
    import time
    import torch
    from hdr2sdr import _abi
    W, H = 256, 128
    p = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
    a = hdr2sdr.Tonemapper(0, p, lattice(65))
    src = synth_frames('smooth', 2, W, H, 10, device='cpu', seed=4).to_torch('cuda')
    dst = hdr2sdr.FrameBatch.empty_torch(2, W, H, 10, 'cuda')
    a.process(src, dst)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(50_000_000)
    torch.cuda.synchronize()
    spin = int(50_000_000 * 0.3 / max(time.perf_counter() - t0, 1e-4))
    try:
        with torch.cuda.stream(side):
            torch.cuda._sleep(spin)
        a.set_option(_abi.OPT_TEST_FAIL_AFTER_LAUNCH, 1)
        with pytest.raises(RuntimeError, match='injected failure'):
            a.process(src, dst, side)                   # queued behind the spin, then reports an error
        t0 = time.perf_counter()
        a.set_params(p.with_(gamma=1.5))
        ta = time.perf_counter() - t0
        torch.cuda.synchronize()
        assert ta > 0.1, f'set_params returned after {ta:.3f} s, before the failed call\'s queued launch ran'
        a.process(src, dst)                             # the hook fires once: the context works on
        torch.cuda.synchronize()
    finally:
        a.close()


def test_two_pass_scratch_serialised_across_streams(tm):
    """The BICUBIC two-pass path uses one per-context scratch plane: two
    launches on two streams from the same thread run one after the other
    (ADVICE r02), so both outputs equal the serial result."""
    import torch
    W, H = 512, 256
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, chroma_filter='bicubic')
    tm.set_params(params)
    tm.set_lut(lattice(65))
    s1 = synth_frames('smooth', 3, W, H, 10, device='cpu', seed=61).to_torch('cuda')
    s2 = synth_frames('uniform', 3, W, H, 10, device='cpu', seed=62).to_torch('cuda')
    want1, want2 = tm(s1).to_numpy().buf, tm(s2).to_numpy().buf
    d1 = hdr2sdr.FrameBatch.empty_torch(3, W, H, 10, 'cuda')
    d2 = hdr2sdr.FrameBatch.empty_torch(3, W, H, 10, 'cuda')
    st1, st2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(3):
        tm.process(s1, d1, st1)
        tm.process(s2, d2, st2)
    torch.cuda.synchronize()
    assert np.array_equal(d1.to_numpy().buf, want1)
    assert np.array_equal(d2.to_numpy().buf, want2)


def test_peak_exchange_and_lp_tone_errors(tm):
    """h2s_peak_stats takes device frames only; h2s_peak_feed rejects
    mismatched arrays; an unknown lp_tone is INVALID_ARG at set_params (the
    ABI validates the raw value, which the Python mirror cannot produce)."""
    from hdr2sdr import _abi
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    host = synth_frames('smooth', 2, 128, 64, 10, device='cpu').to_numpy()
    with pytest.raises(ValueError):
        tm.peak_stats(host)
    with pytest.raises(ValueError):
        tm.feed_peak(np.zeros(3), np.zeros(2))
    fmax, favg = tm.peak_stats(host.to_torch('cuda'))
    assert fmax.shape == favg.shape == (2,) and (fmax >= favg).all() and (favg > 0).all()
    c = params.to_c()
    c.lp_tone = 7
    assert tm._L.h2s_set_params(tm._ctx, ctypes.byref(c)) == _abi.H2S_E_INVALID_ARG
    tm.set_params(params)


@pytest.mark.parametrize('W,H', [(130, 98), (194, 66)])
@pytest.mark.parametrize('tmname', ['hable', 'bt.2390'])
def test_tile_interior_boundaries(tm, W, H, tmname):
    """k_tile addresses a tile from launch-constant lane offsets when its rows
    and its chroma halo lie inside the frame (cy0 >= 1, cy0 + 17 <= ch,
    cx0 + 33 <= cw) and clamps per lane otherwise.  These sizes put tiles
    exactly on each equality (cw = 32k + 1, ch = 16m + 1); rows padded to 16
    bytes send them through the tile kernel (+ k_process for the W % 64
    columns).  Equal to the oracle, and to the tight layout's generic-kernel
    result within the same bound."""
    import ctypes
    import torch
    from hdr2sdr import _abi
    F = 2
    params = hdr2sdr.TonemapParams(tonemapper=tmname, gamma=2.2 if tmname == 'hable' else 1.0)
    got_tight, want, _ = run_both(tm, params, 'smooth', W, H, nframes=F)
    src = synth_frames('smooth', F, W, H, 10, device='cpu', seed=11).to_numpy()
    ls = [(W * 2 + 15) // 16 * 16, (W + 15) // 16 * 16, (W + 15) // 16 * 16]
    fp = H * ls[0] + 2 * (H // 2) * ls[1]

    def desc(buf):
        d = _abi.H2SFrames()
        base = buf.data_ptr()
        d.data[0], d.data[1], d.data[2] = base, base + H * ls[0], base + H * ls[0] + H // 2 * ls[1]
        for p in range(3):
            d.linesize[p], d.frame_pitch[p] = ls[p], fp
        d.width, d.height, d.bits, d.location = W, H, 10, _abi.LOC_DEVICE
        return d

    raw_in = torch.from_numpy(_pack_padded(src.buf, W, H, 10, ls, fp)).cuda()
    raw_out = torch.zeros(F * fp + 64, dtype=torch.uint8, device='cuda')
    di, do = desc(raw_in), desc(raw_out)
    assert tm._L.h2s_query_path(tm._ctx, ctypes.byref(di), ctypes.byref(do)) == _abi.PATH_TILE_TAIL
    tm._check(tm._L.h2s_process(tm._ctx, ctypes.byref(di), ctypes.byref(do), F, None))
    torch.cuda.synchronize()
    got = _unpack_padded(raw_out.cpu().numpy(), F, W, H, 10, ls, fp).astype(np.int64)
    assert_close_int(params, got, want, W, H, src.buf)
    assert_close_int(params, got, got_tight, W, H, src.buf)


def test_option_4_is_reserved(tm):
    """key 4 was H2S_OPT_LP_EXACT in ABI 3.3 (and a failure hook
    before that); since 3.4 it is reserved, so an old client fails loudly."""
    from hdr2sdr import _abi
    with pytest.raises(ValueError, match='reserved'):
        tm.set_option(_abi.OPT_RESERVED_4, 1)
    tm.set_option(_abi.OPT_LP_EXACT, 0)
