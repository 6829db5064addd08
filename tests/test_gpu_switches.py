"""GPU parity for the switchable [EXT] stages and the reference's libplacebo
branch (src/utils.py:392-471).

None of these can be pinned without the bundled ffmpeg / libplacebo: each
switch is a named model in the oracle (oracle/h2s_oracle.c) and in libh2s, so
a box with the real binaries can settle it without a kernel rewrite.  Here the
HIP path must match the oracle's restatement of every switch value, and the
switches must actually change the output."""
import numpy as np
import pytest

import oracle
import hdr2sdr
from hdr2sdr import _abi
from hdr2sdr.synth import synth_frames

from test_gpu_parity import assert_close_int, lattice, run_both

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def tm():
    t = hdr2sdr.Tonemapper(0)
    yield t
    t.close()


def _path(tm, params, W, H):
    src = hdr2sdr.FrameBatch.empty_torch(1, W, H, params.bits_in, 'cuda')
    dst = hdr2sdr.FrameBatch.empty_torch(1, W, H, params.bits_out, 'cuda')
    return tm.query_path(src, dst)


# ---- S6 chroma filter (App. B.4) -------------------------------------------
@pytest.mark.parametrize('kind', ['smooth', 'uniform', 'edges'])
@pytest.mark.parametrize('W,H,bits_out', [(128, 64, 10), (70, 18, 8), (2, 2, 10), (6, 10, 12)])
def test_bicubic_chroma_matches_oracle(tm, W, H, bits_out, kind):
    """Two-pass path: per-pixel chroma to a 4:4:4 scratch, then the 7 x 8-tap
    left/centre-sited bicubic decimation, edge-clamped (tiny frames: every
    tap clamps)."""
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=bits_out, chroma_filter='bicubic')
    got, want, wh = run_both(tm, params, kind, W, H, nframes=2)
    assert_close_int(params, got, want, *wh)
    # pass 1 on the tile kernel wherever the box filter gets it (VERDICT r02
    # item 8: whole 64-pixel tiles, 16-byte rows), the generic two-pass path
    # otherwise
    bic = _path(tm, params, W, H)
    tm.set_params(params.with_(chroma_filter='box'))
    box = _path(tm, params, W, H)
    assert bic == (_abi.PATH_TWO_PASS if box == _abi.PATH_GENERIC else box)


@pytest.mark.parametrize('W,H,bits_out', [(256, 64, 10), (352, 34, 8)])    # whole tiles; tiles + tail
def test_bicubic_tile_pass_equals_generic(tm, W, H, bits_out):
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=bits_out, chroma_filter='bicubic')
    tile, _, _ = run_both(tm, params, 'smooth', W, H, nframes=3)
    assert _path(tm, params, W, H) == (_abi.PATH_TILE if W % 64 == 0 else _abi.PATH_TILE_TAIL)
    tm.set_option(_abi.OPT_FAST_PATH, 0)
    try:
        gen, _, _ = run_both(tm, params, 'smooth', W, H, nframes=3)
    finally:
        tm.set_option(_abi.OPT_FAST_PATH, 1)
    assert_close_int(params, tile, gen, W, H)
    assert (tile == gen).mean() > 0.995


def test_bicubic_taps_are_the_swscale_kernel():
    wx, wy = oracle.chroma_taps()
    assert wx.sum() == pytest.approx(1.0, abs=1e-6) and wy.sum() == pytest.approx(1.0, abs=1e-6)
    assert np.allclose(wx, wx[::-1]) and np.allclose(wy, wy[::-1])      # symmetric about the sited sample
    assert wx[3] == wx.max() and wy[3] == wy[4] == wy.max()             # left-sited / centred
    assert (wx[[0, 6]] < 0).all()                                        # C = 0.6 lobes


def test_chroma_filter_changes_only_chroma(tm):
    """Same kernel family both ways (the generic kernel: the bicubic filter
    has no tile form), so any luma difference would be the filter's."""
    box = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2)
    bic = box.with_(chroma_filter='bicubic')
    tm.set_option(_abi.OPT_FAST_PATH, 0)
    try:
        a, _, _ = run_both(tm, box, 'uniform', 128, 64)
        b, _, _ = run_both(tm, bic, 'uniform', 128, 64)
    finally:
        tm.set_option(_abi.OPT_FAST_PATH, 1)
    ysz = 128 * 64
    assert np.array_equal(a[:, :ysz], b[:, :ysz])
    assert not np.array_equal(a[:, ysz:], b[:, ysz:])


# ---- S6 dither (App. B.4) and S8 expansion (App. B.6) -----------------------
@pytest.mark.parametrize('bits_out', [8, 10, 12])
@pytest.mark.parametrize('mode', ['compat8', 'native'])
def test_ordered_dither_matches_oracle(tm, bits_out, mode):
    params = hdr2sdr.TonemapParams(tonemapper='mobius', gamma=1.4, bits_out=bits_out, mode=mode, dither='ordered')
    got, want, wh = run_both(tm, params, 'smooth', 128, 64)
    assert_close_int(params, got, want, *wh)
    plain, _, _ = run_both(tm, params.with_(dither='none'), 'smooth', 128, 64)
    q = oracle.quant_bits(oracle.params_from(params.to_c()))
    # swscale dithers only its 8-bit output: native 10/12-bit quantisers ignore it
    assert np.array_equal(got, plain) == (q != 8)


@pytest.mark.parametrize('bits_out', [10, 12])
def test_bit_replication_matches_oracle(tm, bits_out):
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=bits_out, expand='replicate')
    got, want, wh = run_both(tm, params, 'ramp', 128, 64)
    assert_close_int(params, got, want, *wh)
    s = bits_out - 8
    v8 = got >> s
    assert np.array_equal(got, (v8 << s) | (v8 >> (8 - s)))           # every code is a replication


@pytest.mark.parametrize('W,H', [(128, 64), (352, 34)])                   # whole tiles; tiles + generic tail (16-B rows)
@pytest.mark.parametrize('kw', [dict(dither='ordered', bits_out=8), dict(dither='ordered', bits_out=10, gamma=1.4),
                                dict(expand='replicate', bits_out=10), dict(expand='replicate', bits_out=12),
                                dict(dither='ordered', expand='replicate', bits_out=12)])
def test_dither_and_replication_run_on_the_tile_kernel(tm, kw, W, H):
    """the S6 dither and S8 bit replication are served by
    k_tile (h2s_query_path TILE) and agree with the oracle and with the
    generic kernel across the tile / tail seam (absolute pixel coordinates
    index the dither matrix on both)."""
    params = hdr2sdr.TonemapParams(**dict(dict(tonemapper='hable', gamma=2.2), **kw))
    got, want, wh = run_both(tm, params, 'smooth', W, H)
    assert_close_int(params, got, want, *wh)
    assert _path(tm, params, W, H) == (_abi.PATH_TILE if W % 64 == 0 else _abi.PATH_TILE_TAIL)
    tm.set_option(_abi.OPT_FAST_PATH, 0)
    try:
        gen, _, _ = run_both(tm, params, 'smooth', W, H)
    finally:
        tm.set_option(_abi.OPT_FAST_PATH, 1)
    assert (got == gen).mean() > 0.995


# ---- the libplacebo branch (src/utils.py:392-471) ---------------------------
LP_CASES = {
    'C3_bt2390': dict(tonemapper='bt.2390'),
    'C3_bt2390_itu_knee': dict(tonemapper='bt.2390', knee_offset=0.5),
    'bt2390_no_black': dict(tonemapper='bt.2390', target_black=0.0),
    'spline': dict(tonemapper='spline'),
    'spline_white100': dict(tonemapper='spline', target_white=100.0),
    'bt2390_gamma13_eq': dict(tonemapper='bt.2390', gamma=1.3),
    'bt2390_8bit': dict(tonemapper='bt.2390', bits_out=8),
    'bt2390_hlg12': dict(tonemapper='bt.2390', bits_in=12, bits_out=12, transfer='arib-std-b67'),
    'bt2390_lut_off_nv12': dict(tonemapper='bt.2390', lut_enabled=False),
    'bt2390_max_rgb': dict(tonemapper='bt.2390', lp_tone='max-rgb'),
    'spline_max_rgb_hlg12': dict(tonemapper='spline', lp_tone='max-rgb', bits_in=12, bits_out=12,
                                 transfer='arib-std-b67'),
    'bt2390_max_rgb_lut_off': dict(tonemapper='bt.2390', lp_tone='max-rgb', lut_enabled=False),
    # libplacebo's own reinhard / hable / mobius (NORM scaling)
    'lp_hable': dict(tonemapper='hable', pipeline='libplacebo'),
    'lp_mobius_max_rgb': dict(tonemapper='mobius', pipeline='libplacebo', lp_tone='max-rgb'),
    'lp_reinhard_hlg12_lut_off': dict(tonemapper='reinhard', pipeline='libplacebo', bits_in=12, bits_out=12,
                                      transfer='arib-std-b67', lut_enabled=False),
    'lp_mobius_gamma13': dict(tonemapper='mobius', pipeline='libplacebo', gamma=1.3),
    # the stage's open options (ABI v3; include/h2s.h enum h2s_lp_range / _dither / _p010)
    'bt2390_range_limited': dict(tonemapper='bt.2390', lp_range='limited'),
    'bt2390_dither_ordered': dict(tonemapper='bt.2390', lp_dither='ordered'),
    'spline_limited_dither_8bit': dict(tonemapper='spline', lp_range='limited', lp_dither='ordered', bits_out=8),
    'bt2390_pq12_p010_keep': dict(tonemapper='bt.2390', bits_in=12, bits_out=10),
    'bt2390_pq12_p010_truncate': dict(tonemapper='bt.2390', bits_in=12, bits_out=10, lp_p010='truncate'),
    'lp_hable_hlg12_p010_truncate_dither': dict(tonemapper='hable', pipeline='libplacebo', bits_in=12, bits_out=12,
                                               transfer='arib-std-b67', lp_p010='truncate', lp_dither='ordered'),
    # the S6 swscale dither (App. B.4) after the branch's eq / 8-bit output:
    # it acts on the final luma quantiser only, never on lut3d's input
    'bt2390_gamma13_eq_sws_dither': dict(tonemapper='bt.2390', gamma=1.3, dither='ordered'),
    'bt2390_8bit_sws_dither': dict(tonemapper='bt.2390', bits_out=8, dither='ordered'),
}


@pytest.mark.parametrize('kind', ['smooth', 'uniform', 'ramp', 'edges'])
@pytest.mark.parametrize('case', sorted(LP_CASES))
def test_libplacebo_branch_matches_oracle(tm, case, kind):
    params = hdr2sdr.TonemapParams(**LP_CASES[case])
    assert params.resolved_pipeline() == 'libplacebo'
    got, want, wh = run_both(tm, params, kind, 128, 64)
    assert_close_int(params, got, want, *wh)
    # every operator of the branch runs on the tile kernel (k_tile<..., LP = 1>),
    # with the LUT on or off
    assert _path(tm, params, 128, 64) == _abi.PATH_TILE


@pytest.mark.parametrize('case', ['C3_bt2390', 'spline', 'bt2390_gamma13_eq', 'bt2390_hlg12', 'bt2390_max_rgb',
                                  'bt2390_lut_off_nv12', 'bt2390_max_rgb_lut_off', 'lp_hable', 'lp_mobius_max_rgb',
                                  'lp_reinhard_hlg12_lut_off', 'bt2390_range_limited', 'bt2390_dither_ordered',
                                  'bt2390_pq12_p010_truncate', 'lp_hable_hlg12_p010_truncate_dither',
                                  'bt2390_gamma13_eq_sws_dither', 'bt2390_8bit_sws_dither'])
def test_libplacebo_tile_equals_generic(tm, case):
    """The two kernels of the libplacebo branch against each other (same
    device, same float32 formulas up to the tile kernel's PQ table): the
    bound of assert_close_int with the generic kernel as the reference."""
    params = hdr2sdr.TonemapParams(**LP_CASES[case])
    host = synth_frames('smooth', 2, 256, 64, params.bits_in, device='cpu', seed=4)
    src = host.to_torch('cuda')
    tm.set_params(params)
    tm.set_lut(lattice(65))
    tile = tm(src).to_numpy().buf.astype(np.int64)
    tm.set_option(_abi.OPT_FAST_PATH, 0)
    try:
        gen = tm(src).to_numpy().buf.astype(np.int64)
    finally:
        tm.set_option(_abi.OPT_FAST_PATH, 1)
    assert_close_int(params, tile, gen, 256, 64, host.to_numpy().buf)
    assert (tile == gen).mean() > 0.99


@pytest.mark.parametrize('kw,min_changed', [
    (dict(lp_range='limited'), 0.5),                          # every code moves towards mid-grey
    (dict(lp_dither='ordered'), 0.02),                        # a fraction of the codes step by one
    (dict(lp_p010='keep', bits_in=12), 0.02),                 # 12-bit input: two low bits kept (default: dropped)
])
def test_libplacebo_options_change_the_output(tm, kw, min_changed):
    base = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_in=kw.get('bits_in', 10))
    src = synth_frames('smooth', 1, 256, 64, base.bits_in, device='cpu', seed=8).to_torch('cuda')
    tm.set_params(base)
    tm.set_lut(lattice(65))
    a = tm(src).to_numpy().buf
    tm.set_params(base.with_(**kw))
    b = tm(src).to_numpy().buf
    assert (a != b).mean() > min_changed


def test_p010_truncate_has_no_effect_on_10bit_input(tm):
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390')
    src = synth_frames('uniform', 1, 128, 64, 10, device='cpu', seed=9).to_torch('cuda')
    tm.set_params(p)
    tm.set_lut(lattice(65))
    a = tm(src).to_numpy().buf
    tm.set_params(p.with_(lp_p010='keep' if p.lp_p010 == 'truncate' else 'truncate'))
    assert np.array_equal(tm(src).to_numpy().buf, a)


def test_lp_tone_ipt_changes_only_coloured_pixels(tm):
    """h2s_lp_tone: IPT and MAX_RGB apply the same curve, so neutral pixels
    (R = G = B) agree within the HPE normalisation's rounding; coloured ones
    differ."""
    W, H = 128, 64
    src = hdr2sdr.FrameBatch.empty_numpy(1, W, H, 10)
    src.y[0] = np.linspace(64, 940, W * H).reshape(H, W).astype(np.uint16)
    src.u[0] = 512
    src.v[0] = 512
    ipt = hdr2sdr.TonemapParams(tonemapper='bt.2390')
    outs = []
    for p in (ipt, ipt.with_(lp_tone='max-rgb')):
        tm.set_params(p)
        tm.set_lut(lattice(65))
        outs.append(tm(src.to_torch('cuda')).to_numpy().buf.astype(np.int64))
    assert np.abs(outs[0] - outs[1]).max() <= 2 and (outs[0] != outs[1]).mean() < 0.01
    col, _, _ = run_both(tm, ipt, 'smooth', W, H)
    col2, _, _ = run_both(tm, ipt.with_(lp_tone='max-rgb'), 'smooth', W, H)
    assert (col != col2).mean() > 0.05


def test_libplacebo_rgba_codes_use_the_full_output_depth(tm):
    """The reference C3 output (rgba -> yuv420p10le, no eq at gamma 1) holds
    10-bit codes that are not multiples of 4; the CPU chain's cannot."""
    lp = hdr2sdr.TonemapParams(tonemapper='bt.2390')
    cpu = lp.with_(pipeline='cpu')
    a, _, _ = run_both(tm, lp, 'smooth', 128, 64)
    b, _, _ = run_both(tm, cpu, 'smooth', 128, 64)
    assert (a % 4 != 0).mean() > 0.5
    assert (b % 4 == 0).all()
    assert oracle.quant_bits(oracle.params_from(lp.to_c())) == 10
    assert oracle.quant_bits(oracle.params_from(lp.with_(gamma=1.3).to_c())) == 8   # eq forces yuv420p


def test_libplacebo_chain_string_selects_the_branch(tm):
    chain = ('[0:v:0]format=p010,hwupload,libplacebo=w=iw:h=ih:tonemapping=bt.2390:colorspace=bt709:'
             'color_primaries=auto:color_trc=bt709:range=tv:peak_detect=1:format=rgba,hwdownload,format=rgba,'
             'lut3d=file=<LUT>:interp=tetrahedral,setparams=color_primaries=bt709:color_trc=bt709:'
             'colorspace=bt709[vout]')
    params, _ = hdr2sdr.parse_filter_chain(chain)
    assert params.pipeline == 'libplacebo' and params.peak_detect
    params = params.with_(peak_detect=False)
    got, want, wh = run_both(tm, params, 'smooth', 128, 64)
    assert_close_int(params, got, want, *wh)


@pytest.mark.parametrize('tmname', ['bt.2390', 'mobius'])
@pytest.mark.parametrize('W,H', [(256, 128), (200, 96)])
def test_libplacebo_dynamic_peak(W, H, tmname):
    """peak_detect=1 (src/utils.py:448) on the libplacebo branch, across calls."""
    from test_peak_detect import sequence
    buf = sequence(W, H)
    params = hdr2sdr.TonemapParams(tonemapper=tmname, peak_detect=True, maxcll=4000.0, pipeline='libplacebo')
    t = hdr2sdr.Tonemapper(0, params, lattice(65))
    got = []
    for a, b in ((0, 2), (2, 6)):
        dst = hdr2sdr.FrameBatch.empty_numpy(b - a, W, H, 10)
        t.process(hdr2sdr.FrameBatch(np.ascontiguousarray(buf[a:b]), W, H, 10), dst)
        got.append(dst.buf)
    t.close()
    knees = []
    want, _ = oracle.process_dynamic(oracle.params_from(params.to_c()), lattice(65), buf, W, H, knees=knees)
    assert_close_int(params, np.concatenate(got).astype(np.int64), want.astype(np.int64), W, H, buf, knees=knees)


# ---- the reference's second pixel gate --------------------------------------
def identity_lattice(n):
    g = np.linspace(0.0, 1.0, n, dtype=np.float64)
    b, gg, r = np.meshgrid(g, g, g, indexing='ij')           # .cube order: red fastest
    return np.stack([r.ravel(), gg.ravel(), b.ravel()], axis=1).astype(np.float32)


@pytest.mark.parametrize('kind,seed', [('smooth', 21), ('ramp', 5)])
def test_gpu_lut_stage_changes_hable_output(kind, seed):
    """TestGpuLutStageActuallyChangesCpuCapableTonemapperOutput
    (test/smoke_test.py:386-435) on the product path: Hable, one 960x540
    HDR10 frame rendered as the reference's preview PNG, with the LUT stage
    vs with that stage a no-op (an identity lattice: the failure the gate
    guards against, "the LUT stage has silently become a no-op"), sampled on
    the 21 x 21 grid (w // 20 steps): the max per-channel difference must be
    >= 30/255 (_MIN_EXPECTED_DIFF, :408).  The reference measured ~61/255
    against libplacebo's own gamut mapping, which is not restated here."""
    from hdr2sdr import preview as PV
    W, H = 960, 540
    src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=seed).to_numpy()
    imgs = []
    for lat in (lattice(65), identity_lattice(65)):
        with PV.Previewer(0, tonemapper='hable', lut_enabled=True, lattice=lat) as pv:
            imgs.append(pv.convert(src, 'iw', 'ih').astype(int))
    xs = np.arange(0, W, max(1, W // 20))
    ys = np.arange(0, H, max(1, H // 20))
    d = np.abs(imgs[0][ys][:, xs] - imgs[1][ys][:, xs])
    assert d.max() >= 30, f'LUT stage changes the Hable output by only {d.max()}/255'


# ---- S1 chroma upsampler edge rule (App. B.2) --------------------------------
@pytest.mark.parametrize('edge', ['zimg', 'replicate', 'mirror'])
@pytest.mark.parametrize('W,H,extra', [
    (128, 64, {}),                                   # k_tile only
    (80, 34, {}),                                    # k_tile + k_process tail (the seam reads column cw)
    (18, 6, {}),                                     # k_process, ragged group
    (2, 2, {}),                                      # 1 x 1 chroma planes
    (128, 64, {'chroma_filter': 'bicubic'}),         # two-pass path
    (128, 64, {'tonemapper': 'bt.2390'}),            # libplacebo branch on k_tile
    (192, 32, {'bits_in': 12, 'bits_out': 12, 'transfer': 'arib-std-b67'}),
])
def test_chroma_edge_matches_oracle(tm, edge, W, H, extra):
    kw = dict(tonemapper='hable', gamma=2.2, chroma_edge=edge)
    kw.update(extra)
    params = hdr2sdr.TonemapParams(**kw)
    for kind in ('uniform', 'edges'):
        got, want, wh = run_both(tm, params, kind, W, H, nframes=2)
        assert_close_int(params, got, want, *wh)


def test_chroma_edge_debug_float_on_tile_path(tm):
    """The tile kernel's own debug instance reads the border rows through
    the same rule (stage 1, linear RGB, mirror)."""
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, chroma_edge='mirror')
    W, H = 128, 64
    src = synth_frames('uniform', 1, W, H, 10, device='cpu', seed=2)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    got = tm.debug_float(src.to_torch('cuda'), 1).astype(np.float64)
    want = oracle.debug_float(oracle.params_from(params.to_c()), lattice(65), src.to_numpy().buf, W, H,
                              1).astype(np.float64)
    rows = [0, H - 1]
    err = np.abs(got[:, rows] - want[:, rows])
    ok = np.isfinite(want[:, rows]) & (np.abs(want[:, rows]) < 1e6)
    assert (err[ok] <= 1e-3 * np.abs(want[:, rows][ok]) + 2e-7).all()


# ---- S3 -> S4 format (App. B.3) ----------------------------------------------
@pytest.mark.parametrize('kw', [dict(tonemapper='hable', gamma=2.2, bits_out=10),
                                dict(tonemapper='mobius', bits_out=10, mode='native'),
                                dict(tonemapper='reinhard', bits_out=8),
                                dict(tonemapper='hable', bits_in=12, bits_out=12, transfer='arib-std-b67')])
@pytest.mark.parametrize('kind', ['smooth', 'uniform', 'edges'])
def test_rgb48_lut_input_matches_oracle(tm, kw, kind):
    params = hdr2sdr.TonemapParams(lut_input='rgb48', **kw)
    got, want, wh = run_both(tm, params, kind, 128, 64)
    assert_close_int(params, got, want, *wh)
    assert _path(tm, params, 128, 64) == _abi.PATH_GENERIC      # the tile kernel models the float path only


def test_rgb48_debug_stage4_matches_oracle(tm):
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, lut_input='rgb48')
    W, H = 128, 64
    src = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=6)
    tm.set_params(params)
    tm.set_lut(lattice(65))
    got = tm.debug_float(src.to_torch('cuda'), 4).astype(np.float64)
    want = oracle.debug_float(oracle.params_from(params.to_c()), lattice(65), src.to_numpy().buf, W, H,
                              4).astype(np.float64)
    d = np.abs(got - want)
    # both are k / 65535.  Where all four corners are exactly 1.0 (the gamut
    # clip saturates large parts of the lattice) the blend is 1.0 or
    # 0.99999994 depending on FMA contraction (fused on the GPU, separate on
    # the oracle's x86 build) and lut3d's truncation maps that to 65535 or
    # 65534: one 16-bit step, invisible after the 8/10-bit quantiser.  A flip
    # of the 16-bit input rounding (an ulp of the GPU's vs libm's powf next to
    # a rounding boundary) moves the coordinate by (N-1)/65535 and the value by
    # a few steps (~2 % of values here).  The 1e-3 float bound holds for all.
    assert (d <= 1e-3 * np.abs(want) + 6e-4).all()
    assert (d < 1.5 / 65535).mean() > 0.95


# H2S_OPT_LP_EXACT (the branch on the generic kernel: stages 1-3 in exact
# arithmetic, h2s_lpx.h, as the oracle's chain_lp_d) over the branch's cases
# without eq (eq after the quantiser spreads a one-step difference) against
# the oracle: every sample within one output step, on whole tiles and on
# tiles + tail columns
@pytest.mark.parametrize('W,H', [(128, 64), (200, 96)])
@pytest.mark.parametrize('kind', ['smooth', 'uniform', 'ramp', 'edges'])
@pytest.mark.parametrize('case', sorted(c for c in LP_CASES if LP_CASES[c].get('gamma', 1.0) == 1.0))
def test_libplacebo_lp_exact_within_one_step(tm, case, kind, W, H):
    params = hdr2sdr.TonemapParams(**LP_CASES[case])
    tm.set_option(_abi.OPT_LP_EXACT, 1)
    try:
        got, want, wh = run_both(tm, params, kind, W, H)
        assert _path(tm, params, W, H) == _abi.PATH_GENERIC
    finally:
        tm.set_option(_abi.OPT_LP_EXACT, 0)
    op = oracle.params_from(params.to_c())
    step = 1 << max(0, params.bits_out - oracle.quant_bits(op))
    d = np.abs(got - want)
    assert d.max(initial=0) <= step, f'max diff {d.max()} > one step ({step}); {(d > step).sum()} samples beyond'
