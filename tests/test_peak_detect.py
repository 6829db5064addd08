"""Dynamic peak for BT.2390 (libplacebo peak_detect=1, src/utils.py:448).

PARITY UNPINNED against libplacebo (not in this image).  The model is stated
in DESIGN.md §4.6 and restated in the oracle: per frame a peak measurement
(the pd_percentile-th percentile of the PQ-encoded max(R,G,B), from a
1024-bin histogram; the maximum at 100) and the mean; an IIR with
coefficient 1 - exp(-1 / pd_smoothing) that a smoothstep over a
pd_scene_low .. pd_scene_high % PQ change of the average bypasses at scene
cuts; the result clamped to [pd_min_peak x SDR white, static peak].
Defaults: vf_libplacebo's options (100 frames, 5.5 / 10 %, 99.995, 1.0);
ROUND2 below is round 2's fixed model (20 frames, 10 / 30 %, maximum, 100
nits).  The GPU path (per-frame stats kernel, then the smoothing and the
per-frame curve records on the device, queued with the conversion) must
match that restatement frame by frame, across calls on one context."""
import math

import numpy as np
import pytest

import oracle
import hdr2sdr
from hdr2sdr.synth import synth_frames


# round 2's fixed model; its 100-nit floor as a fraction of the 203-nit SDR white
ROUND2 = dict(pd_smoothing=20.0, pd_scene_low=10.0, pd_scene_high=30.0, pd_percentile=100.0, pd_min_peak=100.0 / 203.0)


def test_peak_state_first_frame_constant_and_scene_cut():
    st = oracle.PeakState(**{k: v for k, v in ROUND2.items() if k != 'pd_percentile'})
    p0 = st.update(0.6, 0.3, 40.0)
    assert p0 == pytest.approx(oracle.pq_eotf_d(0.6) * 100)
    for _ in range(5):                               # constant input: constant peak
        assert st.update(0.6, 0.3, 40.0) == pytest.approx(p0)
    st.update(0.7, 0.35, 40.0)                       # 5 % PQ change: plain IIR step
    assert st.max == pytest.approx(0.6 + (1 - math.exp(-1 / 20)) * 0.1)
    st.update(0.9, 0.8, 40.0)                        # ~45 % PQ change of the average: scene cut, jump
    assert st.max == pytest.approx(0.9) and st.avg == pytest.approx(0.8)


def test_peak_state_vf_libplacebo_defaults():
    """smoothing_period 100, scene thresholds 5.5 / 10 % PQ of the average"""
    st = oracle.PeakState()
    st.update(0.6, 0.3, 40.0)
    st.update(0.7, 0.33, 40.0)                       # 3 % change: plain IIR step, 1 - exp(-1/100)
    assert st.max == pytest.approx(0.6 + (1 - math.exp(-1 / 100)) * 0.1)
    st.update(0.9, 0.6, 40.0)                        # 27 % > 10 %: full bypass
    assert st.max == pytest.approx(0.9) and st.avg == pytest.approx(0.6)
    a = 1 - math.exp(-1 / 100)
    st.update(0.5, 0.6 + 0.0775, 40.0)               # 7.75 %: half-way through the band, smoothstep 0.5
    assert st.max == pytest.approx(0.9 + (a + (1 - a) * 0.5) * (0.5 - 0.9))


def test_peak_clamps_to_minimum_and_static_peak():
    st = oracle.PeakState()
    assert st.update(0.1, 0.05, 10.0) == pytest.approx(2.03)   # minimum_peak 1.0 x the 203-nit SDR white
    st = oracle.PeakState(**ROUND2)
    assert st.update(0.1, 0.05, 10.0) == pytest.approx(1.0)    # round 2: 100 nits
    st = oracle.PeakState()
    assert st.update(0.95, 0.5, 10.0) == 10.0                  # above the static peak -> static


def test_oracle_percentile_cuts_isolated_highlights():
    """99.995 % of 256 x 256 pixels cuts the brightest 3.3 pixels' worth, so
    two isolated super-bright pixels do not set the peak; 100 = the maximum."""
    fb = _flat_frame(64 + round(0.5 * 876), W=256, H=256)
    fb.y[0, 0, :2] = 940                             # two pixels at E = 1
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True)
    mx, _ = oracle.peak_stats(oracle.params_from(p.to_c()), fb.buf, 256, 256)
    assert mx[0] < 0.51
    mx, _ = oracle.peak_stats(oracle.params_from(p.with_(pd_percentile=100.0).to_c()), fb.buf, 256, 256)
    assert mx[0] == pytest.approx(1.0)


def _flat_frame(code_y, code_c=512, W=64, H=32):
    fb = hdr2sdr.FrameBatch.empty_numpy(1, W, H, 10)
    fb.y[...] = code_y
    fb.u[...] = code_c
    fb.v[...] = code_c
    return fb


def test_oracle_peak_stats_neutral_frame():
    code = 64 + round(0.5 * 876)                     # E = 0.5 on every channel
    p = oracle.params_from(hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True).to_c())
    mx, avg = oracle.peak_stats(p, _flat_frame(code).buf, 64, 32)
    assert mx[0] == pytest.approx((code - 64) / 876, abs=1e-9) and avg[0] == pytest.approx(mx[0])


def test_libplacebo_chain_turns_peak_detect_on():
    params, _ = hdr2sdr.parse_filter_chain(
        'format=p010,hwupload,libplacebo=w=iw:h=ih:tonemapping=bt.2390:colorspace=bt709:peak_detect=1:format=rgba,'
        'hwdownload,format=rgba,lut3d=file=<LUT>:interp=tetrahedral')
    assert params.peak_detect and params.tonemapper == 'bt.2390'


def sequence(W=256, H=128):
    """6 frames of different brightness with a scene cut at frame 3."""
    frames = []
    for i, k in enumerate((0.62, 0.62, 0.66, 0.30, 0.30, 0.64)):
        f = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=40 + i).to_numpy()
        f.y[...] = (64 + (f.y.astype(np.float64) - 64) * k).round().astype(np.uint16)
        f.u[...] = (512 + (f.u.astype(np.float64) - 512) * k).round().astype(np.uint16)
        f.v[...] = (512 + (f.v.astype(np.float64) - 512) * k).round().astype(np.uint16)
        frames.append(f.buf)
    return np.concatenate(frames)


@pytest.mark.gpu
@pytest.mark.parametrize('model', ['vf_libplacebo', 'round2'])
@pytest.mark.parametrize('pipeline', ['cpu', 'libplacebo'])  # cpu: the tile kernel's per-frame curve records
@pytest.mark.parametrize('tmname', ['bt.2390', 'spline'])   # spline also takes its knee from the average
@pytest.mark.parametrize('W,H', [(256, 128), (192, 96), (200, 96)])   # fast path (blocks within / across frames), + tail
def test_gpu_dynamic_peak_matches_oracle_across_calls(W, H, tmname, pipeline, model):
    from test_gpu_parity import assert_close_int, lattice
    buf = sequence(W, H)
    params = hdr2sdr.TonemapParams(tonemapper=tmname, peak_detect=True, maxcll=4000.0, pipeline=pipeline,
                                   **(ROUND2 if model == 'round2' else {}))
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    got = []
    for a, b in ((0, 2), (2, 5), (5, 6)):            # the state carries across calls
        src = hdr2sdr.FrameBatch(np.ascontiguousarray(buf[a:b]), W, H, 10)
        dst = hdr2sdr.FrameBatch.empty_numpy(b - a, W, H, 10)
        tm.process(src, dst)
        got.append(dst.buf)
    state = tm.peak_state()
    tm.close()
    got = np.concatenate(got).astype(np.int64)
    knees = []
    want, peaks = oracle.process_dynamic(oracle.params_from(params.to_c()), lattice(65), buf, W, H, knees=knees)
    # the peak really moves (under vf_libplacebo's defaults the darker frames
    # sit at the minimum peak, 1.0 x the 203-nit white)
    assert len(set(round(p, 3) for p in peaks)) >= (3 if model == 'round2' else 2)
    assert state['frames'] == 6 and state['peak'] == pytest.approx(peaks[-1], rel=1e-4)
    assert_close_int(params, got, want.astype(np.int64), W, H, buf, knees=knees)


@pytest.mark.gpu
@pytest.mark.parametrize('pipeline', ['cpu', 'libplacebo'])
@pytest.mark.parametrize('W,H', [(256, 128), (200, 96)])   # pipelined schedule; tail width keeps the serial one
def test_gpu_dynamic_peak_chunked_schedule_is_identical(W, H, pipeline):
    """The pipelined dynamic-peak schedule (statistics of chunk j + 1 on
    their own stream beside chunk j's conversion; chunks converted on two
    streams, H2S_OPT_TEST_PEAK_CHUNK frames each, ragged last chunk included)
    gives the unchunked schedule's output and state bit for bit, across calls,
    and matches the oracle's sequential flow."""
    import torch
    from hdr2sdr import _abi
    from test_gpu_parity import assert_close_int, lattice
    seq = sequence(W, H)
    buf = np.concatenate([seq, seq[::-1]])           # 12 frames, three scene cuts
    n = buf.shape[0]
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True, maxcll=4000.0, pipeline=pipeline)
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    src = hdr2sdr.FrameBatch(torch.from_numpy(np.ascontiguousarray(buf)).cuda(), W, H, 10)
    dst = hdr2sdr.FrameBatch.empty_torch(n, W, H, 10, 'cuda')
    runs = {}
    for chunk in (0, 1, 4, 5, 12):
        tm.set_option(_abi.OPT_TEST_PEAK_CHUNK, chunk)
        tm.reset_peak()
        outs = []
        for _ in range(2):                           # the state carries into the second call
            tm.process(src, dst)
            torch.cuda.synchronize()
            outs.append(dst.buf.cpu().numpy().copy())
        runs[chunk] = (outs, tm.peak_state())
    tm.close()
    for chunk in (1, 4, 5, 12):
        assert runs[chunk][1] == runs[0][1], chunk
        for a, b in zip(runs[chunk][0], runs[0][0]):
            assert np.array_equal(a, b), chunk
    knees = []
    want, _ = oracle.process_dynamic(oracle.params_from(params.to_c()), lattice(65), buf, W, H, knees=knees)
    assert_close_int(params, runs[4][0][0].astype(np.int64), want.astype(np.int64), W, H, buf, knees=knees)


@pytest.mark.gpu
@pytest.mark.parametrize('kw', [dict(chroma_filter='bicubic'), dict(gamma=1.3, dither='ordered', lp_dither='ordered'),
                                dict(lp_range='limited', bits_out=8)])
def test_gpu_dynamic_peak_with_switches_matches_oracle(kw):
    """Dynamic peak (per-frame curve records) together with the two-pass
    BICUBIC chroma (one launch pair per frame), the two dithers with eq, and
    range=tv at an 8-bit output, against the oracle's sequential flow."""
    from test_gpu_parity import assert_close_int, lattice
    W, H = 200, 96
    buf = sequence(W, H)
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True, maxcll=4000.0, **kw)
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    src = hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 10)
    dst = hdr2sdr.FrameBatch.empty_numpy(buf.shape[0], W, H, params.bits_out)
    tm.process(src, dst)
    tm.close()
    knees = []
    want, _ = oracle.process_dynamic(oracle.params_from(params.to_c()), lattice(65), buf, W, H, knees=knees)
    assert_close_int(params, dst.buf.astype(np.int64), want.astype(np.int64), W, H, buf, knees=knees)


def _saturated_frames(W, H):
    """Frames with pixels at E > 1 (Y' code 1023: PQ(max R,G,B) clamps to 1
    exactly, the histogram's top edge): a band of whole rows (statistics units
    inside one bin) and every fifth column (units spanning bins), each beside
    E = 0.5."""
    a = _flat_frame(64 + round(0.5 * 876), W=W, H=H)
    a.y[0, : H // 5, :] = 1023
    b = _flat_frame(64 + round(0.5 * 876), W=W, H=H)
    b.y[0, :, ::5] = 1023
    return np.concatenate([a.buf, b.buf])


@pytest.mark.gpu
@pytest.mark.parametrize('pct', [float('nan'), 90.0, 100.0])   # nan: vf_libplacebo's 99.995
@pytest.mark.parametrize('W,H', [(256, 128), (200, 96)])       # quad form; row / generic form
def test_gpu_peak_stats_equal_the_oracle(W, H, pct):
    """h2s_peak_stats (the per-frame percentile measurement and mean) against
    the oracle's, on the sequence and on frames with saturated pixels, whose
    PQ value 1 sits on the histogram's top edge."""
    import torch
    from test_gpu_parity import lattice
    buf = np.concatenate([sequence(W, H), _saturated_frames(W, H)])
    kw = {} if math.isnan(pct) else dict(pd_percentile=pct)
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True, maxcll=4000.0, **kw)
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    fmax, favg = tm.peak_stats(hdr2sdr.FrameBatch(torch.from_numpy(buf).cuda(), W, H, 10))
    tm.close()
    mx, avg = oracle.peak_stats(oracle.params_from(params.to_c()), buf, W, H)
    np.testing.assert_allclose(fmax, mx, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(favg, avg, rtol=1e-5, atol=1e-6)
    if pct == 90.0:          # a fifth of the pixels saturate: the 90th percentile is in the top bin
        assert (fmax[-2:] > 1023 / 1024).all()


@pytest.mark.gpu
def test_gpu_peak_reset_restarts_the_sequence():
    from test_gpu_parity import lattice
    buf = sequence()
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True, maxcll=4000.0)
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    one = hdr2sdr.FrameBatch(np.ascontiguousarray(buf[3:4]), 256, 128, 10)
    out_a = hdr2sdr.FrameBatch.empty_numpy(1, 256, 128, 10)
    tm.process(one, out_a)                             # first frame of a sequence
    tm.process(hdr2sdr.FrameBatch(np.ascontiguousarray(buf[:3]), 256, 128, 10),
               hdr2sdr.FrameBatch.empty_numpy(3, 256, 128, 10))
    tm.reset_peak()
    out_b = hdr2sdr.FrameBatch.empty_numpy(1, 256, 128, 10)
    tm.process(one, out_b)
    assert tm.peak_state()['frames'] == 1
    assert np.array_equal(out_a.buf, out_b.buf)
    tm.close()


@pytest.mark.gpu
@pytest.mark.parametrize('W,H', [(204, 96), (256, 64)])     # scalar stats + tail, streaming stats
def test_gpu_dynamic_peak_hlg12(W, H):
    """12-bit HLG source (C5's input format) under peak detection: the stats
    take the inverse OETF + OOTF path; both stats kernels and the tail."""
    from test_gpu_parity import assert_close_int, lattice
    buf = synth_frames('smooth', 4, W, H, 12, device='cpu', seed=77).to_numpy().buf
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True, transfer='arib-std-b67',
                                   bits_in=12, bits_out=12, pipeline='cpu')
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    src = hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 12)
    dst = hdr2sdr.FrameBatch.empty_numpy(4, W, H, 12)
    tm.process(src, dst)
    state = tm.peak_state()
    tm.close()
    want, peaks = oracle.process_dynamic(oracle.params_from(params.to_c()), lattice(65), buf, W, H)
    assert state['frames'] == 4 and state['peak'] == pytest.approx(peaks[-1], rel=1e-4)
    assert_close_int(params, dst.buf.astype(np.int64), want.astype(np.int64), W, H)


@pytest.mark.gpu
@pytest.mark.parametrize('tmname', ['bt.2390', 'spline'])
def test_gpu_sharded_peak_state_equals_sequential(tmname):
    """hdr2sdr.dist.sync_peak_state's device half: a second context that is
    fed the statistics of the frames before its range (h2s_peak_stats ->
    h2s_peak_feed) converts its frames bit-identically to one context that
    walked the whole sequence, and ends in the same smoothing state."""
    from test_gpu_parity import lattice
    W, H = 256, 128
    buf = sequence(W, H)
    params = hdr2sdr.TonemapParams(tonemapper=tmname, peak_detect=True, maxcll=4000.0)
    src = hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 10).to_torch('cuda')
    seq = hdr2sdr.Tonemapper(0, params, lattice(65))
    want = seq(src).to_numpy().buf
    state = seq.peak_state()
    fmax, favg = seq.peak_stats(src)
    seq.close()
    shard = hdr2sdr.FrameBatch(np.ascontiguousarray(buf[3:]), W, H, 10).to_torch('cuda')
    r1 = hdr2sdr.Tonemapper(0, params, lattice(65))
    r1.feed_peak(fmax[:3], favg[:3])
    got = r1(shard).to_numpy().buf
    assert np.array_equal(got, want[3:])
    assert r1.peak_state() == state
    r1.close()


def _spin_cycles(seconds):
    """torch's spin kernel argument for ~seconds on this device (its cycle
    counter's rate, calibrated)."""
    import time
    import torch
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(50_000_000)
    torch.cuda.synchronize()
    return int(50_000_000 * seconds / max(time.perf_counter() - t0, 1e-4))


@pytest.mark.gpu
@pytest.mark.parametrize('W,tmname', [(256, 'bt.2390'), (200, 'spline')])   # tile only; tile + generic tail
def test_gpu_dynamic_peak_call_is_asynchronous(W, tmname):
    """with peak_detect, h2s_process queues the
    statistics, the smoothing and curve records (on the device) and the
    conversion on its stream and returns, as include/h2s.h promises for
    device frames: queued behind a ~0.3 s spin kernel on the same stream the
    call returns long before the spin ends, and the output, the smoothing
    state and the peak equal a call made on an idle stream."""
    import time
    import torch
    from test_gpu_parity import lattice
    H = 128
    buf = sequence(W, H)
    params = hdr2sdr.TonemapParams(tonemapper=tmname, peak_detect=True, maxcll=4000.0)
    src = hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 10).to_torch('cuda')
    ref = hdr2sdr.Tonemapper(0, params, lattice(65))
    want = ref(src).to_numpy().buf
    want_state = ref.peak_state()
    ref.close()
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    dst = hdr2sdr.FrameBatch.empty_torch(buf.shape[0], W, H, 10, 'cuda')
    side = torch.cuda.Stream()
    spin = _spin_cycles(0.3)
    try:
        with torch.cuda.stream(side):
            torch.cuda._sleep(spin)
        t0 = time.perf_counter()
        tm.process(src, dst, side)
        t_call = time.perf_counter() - t0
        busy = not side.query()          # the spin (and the conversion behind it) still running
        torch.cuda.synchronize()
        assert t_call < 0.1 and busy, f'h2s_process(peak_detect) blocked the host for {t_call:.3f} s'
        assert np.array_equal(dst.to_numpy().buf, want)
        assert tm.peak_state() == want_state
    finally:
        tm.close()


@pytest.mark.gpu
def test_gpu_preview_restores_the_contexts_peak_state():
    """a preview on a context that is in the middle of a
    dynamic-peak conversion starts each preview frame from a fresh state (the
    reference's per-frame ffmpeg runs) and leaves the context's own state as
    it found it, so the conversion continues as if no preview had run."""
    import ctypes
    from hdr2sdr import _abi
    from test_gpu_parity import lattice
    W, H = 256, 128
    buf = sequence(W, H)
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True, bits_out=8, maxcll=4000.0)
    seq = hdr2sdr.Tonemapper(0, params, lattice(65))
    want = seq(hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 10)).buf
    seq.close()
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    a = tm(hdr2sdr.FrameBatch(np.ascontiguousarray(buf[:3]), W, H, 10)).buf
    before = tm.peak_state()
    rgb = np.empty((2, H, W, 3), np.uint8)
    d = hdr2sdr.FrameBatch(np.ascontiguousarray(buf[3:5]), W, H, 10).descriptor()
    L = _abi.lib()
    rc = L.h2s_preview_rgb24_batch(tm._ctx, ctypes.byref(d), 2, rgb.ctypes.data, 3 * W, 3 * W * H, W, H, 1.0,
                                   _abi.LOC_HOST, None)
    assert rc == 0, L.h2s_last_error(tm._ctx)
    assert tm.peak_state() == before
    b = tm(hdr2sdr.FrameBatch(np.ascontiguousarray(buf[3:]), W, H, 10)).buf
    tm.close()
    assert np.array_equal(np.concatenate([a, b]), want)


@pytest.mark.gpu
def test_gpu_preview_restores_the_peak_state_when_it_fails():
    """a preview whose per-frame conversion fails after its
    launch (the H2S_OPT_TEST_FAIL_AFTER_LAUNCH hook) still restores the
    context's own peak state before returning the error, so the sequence
    continues as if no preview had run."""
    import ctypes
    from hdr2sdr import _abi
    from test_gpu_parity import lattice
    W, H = 256, 128
    buf = sequence(W, H)
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', peak_detect=True, bits_out=8, maxcll=4000.0)
    seq = hdr2sdr.Tonemapper(0, params, lattice(65))
    want = seq(hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 10)).buf
    seq.close()
    tm = hdr2sdr.Tonemapper(0, params, lattice(65))
    a = tm(hdr2sdr.FrameBatch(np.ascontiguousarray(buf[:3]), W, H, 10)).buf
    before = tm.peak_state()
    rgb = np.empty((2, H, W, 3), np.uint8)
    d = hdr2sdr.FrameBatch(np.ascontiguousarray(buf[3:5]), W, H, 10).descriptor()
    L = _abi.lib()
    tm.set_option(_abi.OPT_TEST_FAIL_AFTER_LAUNCH, 1)
    rc = L.h2s_preview_rgb24_batch(tm._ctx, ctypes.byref(d), 2, rgb.ctypes.data, 3 * W, 3 * W * H, W, H, 1.0,
                                   _abi.LOC_HOST, None)
    assert rc == _abi.H2S_E_HIP and b'injected failure' in L.h2s_last_error(tm._ctx)
    assert tm.peak_state() == before
    b = tm(hdr2sdr.FrameBatch(np.ascontiguousarray(buf[3:]), W, H, 10)).buf
    tm.close()
    assert np.array_equal(np.concatenate([a, b]), want)
