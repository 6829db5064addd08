"""Drop-in planner (hdr2sdr.plan) against the reference's own build() argv
(tests/golden/filter_chains.json, captured by tests/golden/make_golden.py),
plus the pipe executor's mechanics with stand-in decode/encode processes."""
import json
import os
import sys

import numpy as np
import pytest

from hdr2sdr import plan as P

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'filter_chains.json')))
PROPS10 = {'width': 3840, 'height': 2160, 'bit_depth': 10, 'color_transfer': 'smpte2084', 'frame_rate': 24.0}
PROPS12 = dict(PROPS10, bit_depth=12, color_transfer='arib-std-b67', width=7680, height=4320)

CASES = {  # config -> (tonemapper, gamma, bits_out, lut)
    'C1': ('reinhard', 1.0, 10, True), 'C2': ('hable', 2.2, 10, True), 'C3': ('bt.2390', 1.0, 10, True),
    'C4': ('mobius', 1.0, 10, True), 'C5': ('hable', 1.0, 12, True), 'default8': ('mobius', 1.0, 8, True),
    'gamma05': ('hable', 0.5, 8, True),
}


@pytest.mark.parametrize('cfg', sorted(CASES))
def test_plan_from_reference_argv(cfg):
    argv = GOLD[cfg]['argv']
    props = PROPS12 if cfg == 'C5' else PROPS10
    pl = P.plan_from_argv(argv, props, hdr={'maxcll': 1000.0})
    tm, gamma, bits_out, lut = CASES[cfg]
    p = pl.params
    assert (p.tonemapper, p.gamma, p.bits_out, p.lut_enabled) == (tm, gamma, bits_out, lut)
    assert p.bits_in == props['bit_depth'] and p.maxcll == 1000.0
    assert p.transfer == ('arib-std-b67' if cfg == 'C5' else 'smpte2084')
    # decode: raw planar frames of the source depth on stdout
    assert pl.decode[-5:] == ['-f', 'rawvideo', '-pix_fmt', P.PIPE_PIX_FMT[props['bit_depth']], '-']
    assert pl.decode[pl.decode.index('-i') + 1] == 'in.mkv'
    # encode: pipe input 0, original file input 1, then EVERY option the
    # reference's build() chose after its filter graph, in order, with
    # '-map [vout]' dropped and input-0 stream maps moved to input 1
    enc = pl.encode
    assert enc[enc.index('-f') + 1] == 'rawvideo' and enc[enc.index('-s') + 1] == f"{props['width']}x{props['height']}"
    assert enc[enc.index('-i') + 1] == '-' and enc[enc.index('-i', enc.index('-i') + 1) + 1] == 'in.mkv'
    ref_tail = argv[argv.index('-filter_complex') + 2:]
    ref_tail = [t for k, t in enumerate(ref_tail) if not (t == '[vout]' or (t == '-map' and ref_tail[k + 1] == '[vout]'))]
    expect = [('1' + t[1:] if t.startswith('0:') else t) for t in ref_tail]
    expect = ['1' if (t == '0' and k and expect[k - 1] == '-map_metadata') else t for k, t in enumerate(expect)]
    # the BT.709 tags are inserted just before the output path
    tail = enc[enc.index('0:v:0') + 1:]
    o = tail.index('out.mkv')
    assert tail[o - len(P.BT709_TAGS):o] == P.BT709_TAGS
    assert tail[:o - len(P.BT709_TAGS)] + tail[o:] == expect
    assert pl.output_path == 'out.mkv'
    assert enc[enc.index('-pix_fmt') + 1] == P.PIPE_PIX_FMT[bits_out]


def test_plan_drops_pre_input_vulkan_args():
    pl = P.plan_from_argv(GOLD['C3']['argv'], PROPS10)
    assert '-init_hw_device' not in pl.decode + pl.encode
    assert pl.params.tonemapper == 'bt.2390' and pl.params.desat == 0.0


def test_plan_rejects_non_conversion_argv():
    with pytest.raises(ValueError):
        P.plan_from_argv(['ffmpeg', '-i', 'a.mkv', 'b.mkv'], PROPS10)
    bad = list(GOLD['C2']['argv'])
    bad[bad.index('-pix_fmt') + 1] = 'rgb24'
    with pytest.raises(ValueError):
        P.plan_from_argv(bad, PROPS10)
    with pytest.raises(ValueError):
        P.plan_from_argv(GOLD['C2']['argv'], dict(PROPS10, bit_depth=8))
    with pytest.raises(ValueError):
        P.plan_from_argv(GOLD['C2']['argv'], dict(PROPS10, color_transfer='bt709'))


RULES = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'request_rules.json')))


@pytest.mark.parametrize('profile', [5, 8])
def test_plan_refuses_dolby_vision_profile5(profile):
    """the reference sends a Dolby Vision profile 5
    source to libplacebo because libplacebo applies its RPU
    (src/ffmpeg_command.py:100-106, :117-128); the rawvideo pipe drops the
    RPU, so plan_from_argv refuses the argv build() made for it (the caller
    keeps the reference command).  Profile 8 (HDR10-compatible base layer)
    goes through.  The argv is the reference's C3 command with the filter
    graph build() produced for the captured DoVi request."""
    from hdr2sdr import chain as C
    case = next(c for c in RULES['cases'] if c.get('props', {}).get('dovi_profile') == profile
                and 'filter_complex' in c and c['pix_fmt'] == 'yuv420p10le')
    argv = list(GOLD['C3']['argv'])
    argv[argv.index('-filter_complex') + 1] = case['filter_complex']
    props = dict(PROPS10, **case['props'])
    if profile == 5:
        with pytest.raises(ValueError) as e:
            P.plan_from_argv(argv, props)
        assert str(e.value) == C.DOVI_P5_ERROR
        assert 'libplacebo=' in case['filter_complex']   # the reference's routing
    else:
        assert P.plan_from_argv(argv, props).params.resolved_pipeline() == 'cpu'


def test_lut_path_unescape():
    from hdr2sdr.lut import unescape_filter_path
    assert unescape_filter_path('C\\\\:/Program Files/app/luts/rec2020_to_rec709.cube') == \
        'C:/Program Files/app/luts/rec2020_to_rec709.cube'


class _FakeTonemapper:
    """Stand-in GPU stage for the pump mechanics: out = (in >> 2) << 2."""

    def __init__(self):
        self.calls = []

    def process(self, src, dst, stream=None, nframes=None):
        self.calls.append(nframes)
        dst.buf[:nframes] = (src.buf[:nframes] >> 2) << 2


def _fake_pipes(pl, tmp_path, frames):
    raw = tmp_path / 'in.raw'
    frames.tofile(raw)
    out = tmp_path / 'out.raw'
    pl.decode = [sys.executable, '-c', f'import sys; sys.stdout.buffer.write(open({str(raw)!r}, "rb").read())']
    pl.encode = [sys.executable, '-c',
                 f'import sys; d = sys.stdin.buffer.read(); open({str(out)!r}, "wb").write(d); '
                 f'sys.stderr.write("frame= 3 fps=0.0 q=-0.0 size=0kB time=00:00:00.12 bitrate=N/A\\n")']
    return out


@pytest.mark.parametrize('nframes,batch', [(5, 2), (4, 4), (1, 8), (0, 3)])
def test_pipe_executor_mechanics(tmp_path, nframes, batch):
    pl = P.plan_from_argv(GOLD['C2']['argv'], dict(PROPS10, width=64, height=32))
    rng = np.random.default_rng(nframes)
    frames = rng.integers(64, 940, size=(nframes, 64 * 32 * 3 // 2), dtype=np.uint16)
    out = _fake_pipes(pl, tmp_path, frames)
    tm = _FakeTonemapper()
    proc = P.H2SProcess(pl, tm, batch=batch)
    lines = list(proc.stderr)
    assert proc.wait(timeout=60) == 0
    assert any('time=00:00:00.12' in ln for ln in lines)      # monitor_progress's regex source
    got = np.fromfile(out, dtype=np.uint16).reshape(nframes, 64 * 32 * 3 // 2)
    assert np.array_equal(got, (frames >> 2) << 2)
    assert proc.frames == nframes and sum(tm.calls) == nframes


@pytest.mark.parametrize('depth', [1, 3])
def test_pipe_executor_keeps_frame_order_with_read_ahead(tmp_path, depth):
    """The decoder-side reader fills up to `depth` slots ahead of the GPU
    stage; frames still reach the encoder in decode order."""
    pl = P.plan_from_argv(GOLD['C2']['argv'], dict(PROPS10, width=64, height=32))
    nframes = 23
    frames = np.arange(nframes, dtype=np.uint16)[:, None] * 8 + np.zeros((1, 64 * 32 * 3 // 2), np.uint16)
    out = _fake_pipes(pl, tmp_path, frames)
    tm = _FakeTonemapper()
    proc = P.H2SProcess(pl, tm, batch=2, depth=depth)
    list(proc.stderr)
    assert proc.wait(timeout=60) == 0
    got = np.fromfile(out, dtype=np.uint16).reshape(nframes, -1)
    assert np.array_equal(got, frames)
    assert tm.calls == [2] * 11 + [1]


def test_pipe_executor_reports_gpu_failure(tmp_path):
    pl = P.plan_from_argv(GOLD['C2']['argv'], dict(PROPS10, width=64, height=32))
    _fake_pipes(pl, tmp_path, np.zeros((2, 64 * 32 * 3 // 2), np.uint16))

    class Boom:
        def process(self, *a, **k):
            raise RuntimeError('libh2s error -3: device lost')
    proc = P.H2SProcess(pl, Boom(), batch=1)
    list(proc.stderr)
    assert proc.wait(timeout=60) == 1 and isinstance(proc.error, RuntimeError)


@pytest.mark.gpu
@pytest.mark.parametrize('cfg', ['C2', 'default8', 'C5', 'C3'])
def test_planned_conversion_matches_oracle(tmp_path, cfg):
    """The whole drop-in: reference argv -> plan -> decode pipe -> libh2s
    (HIP) -> encode pipe; the encoded bytes equal the oracle's chain."""
    import oracle
    from hdr2sdr.synth import synth_frames
    from test_gpu_parity import assert_close_int, lattice
    W, H, N = 128, 64, 5
    props = dict(PROPS12 if cfg == 'C5' else PROPS10, width=W, height=H)
    pl = P.plan_from_argv(GOLD[cfg]['argv'], props, hdr={'maxcll': 1000.0})
    src = synth_frames('smooth', N, W, H, pl.params.bits_in, device='cpu', seed=5).to_numpy()
    out = _fake_pipes(pl, tmp_path, src.buf)
    proc = P.start(pl, device=0, batch=2)
    list(proc.stderr)
    assert proc.wait(timeout=120) == 0 and proc.error is None and proc.frames == N
    dt = np.uint8 if pl.params.bits_out == 8 else np.uint16
    got = np.fromfile(out, dtype=dt).reshape(N, -1).astype(np.int64)
    op = oracle.params_from(pl.params.to_c())
    knees = None
    if pl.params.peak_detect:      # C3: libplacebo peak_detect=1 -> detected, smoothed peak
        knees = []
        want = oracle.process_dynamic(op, lattice(65), src.buf, W, H, knees=knees)[0].astype(np.int64)
    else:
        want = oracle.process(op, lattice(65), src.buf, W, H).astype(np.int64)
    assert_close_int(pl.params, got, want, W, H, src.buf, knees=knees)
