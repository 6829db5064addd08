"""BASELINE.json's five configurations on the HIP path, first in the `-m gpu`
run (this file sorts before every other test module), so that a `-x` stop
later in the suite cannot hide them:

* full-size frames of C1-C5 (1080p Reinhard + 33^3 at 8 bits; 4K Hable +
  65^3 + eq 2.2; 4K BT.2390 on the libplacebo branch; 4K Mobius; 8K 12-bit
  HLG Hable 12-bit out) against the CPU oracle, integer tolerance as
  tests/test_gpu_parity.py's assert_close_int;
* the tile kernel's own float stages (k_tile debug instances, the arithmetic
  h2s_process runs) for the same configurations at 1e-3 relative, per stage.

Reference anchors: the CPU chain src/utils.py:38-42 (C1, C2, C4, C5), the
libplacebo chain src/utils.py:392-471 (C3), the output formats
src/ffmpeg_command.py:355-360."""
import pytest

import hdr2sdr

from test_gpu_parity import assert_close_int, check_float_stage, run_both

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def tm():
    t = hdr2sdr.Tonemapper(0)
    yield t
    t.close()


@pytest.mark.parametrize('name,kw,W,H,nframes', [
    ('C1_1080p_reinhard_33_8bit', dict(tonemapper='reinhard', gamma=1.0, bits_out=8), 1920, 1080, 1),
    ('C2_4k_hable_g22', dict(tonemapper='hable', gamma=2.2, bits_out=10), 3840, 2160, 2),
    ('C3_4k_bt2390', dict(tonemapper='bt.2390', gamma=1.0, bits_out=10), 3840, 2160, 1),
    ('4k_spline', dict(tonemapper='spline', gamma=1.0, bits_out=10), 3840, 2160, 1),
    ('C4_4k_mobius', dict(tonemapper='mobius', gamma=1.0, bits_out=10), 3840, 2160, 1),
    ('C5_8k_hlg12_hable', dict(tonemapper='hable', gamma=1.0, bits_in=12, bits_out=12, transfer='arib-std-b67'),
     7680, 4320, 1),
])
def test_full_size_configs(tm, name, kw, W, H, nframes):
    params = hdr2sdr.TonemapParams(**kw)
    lut_n = 33 if name.startswith('C1') else 65
    got, want, wh = run_both(tm, params, 'smooth', W, H, nframes=nframes, lut_n=lut_n)
    assert_close_int(params, got, want, *wh, lut_n=lut_n)


def test_full_size_uniform_worst_case(tm):
    params = hdr2sdr.TonemapParams(tonemapper='hable', gamma=2.2, bits_out=10)
    got, want, _ = run_both(tm, params, 'uniform', 3840, 2160, nframes=1)
    assert_close_int(params, got, want, 3840, 2160)


# the BASELINE configurations among test_gpu_parity.FLOAT_CFGS, on the tile kernel
@pytest.mark.parametrize('stage', [1, 2, 3, 4, 5])
@pytest.mark.parametrize('kind', ['ramp', 'uniform'])
@pytest.mark.parametrize('cfg', ['C2_hable_pq10', 'C3_bt2390_libplacebo', 'C4_mobius_native', 'C5_hable_hlg12'])
def test_tile_kernel_float_stages(tm, cfg, kind, stage):
    check_float_stage(tm, 'k_tile', cfg, kind, stage)


def test_c3_as_the_reference_runs_it_4k_sequence(tm):
    """C3 exactly as the reference's build() emits it for a BT.2390 request
    with GPU tone mapping on (tests/golden/filter_chains.json C3:
    format=p010,hwupload,libplacebo=...:peak_detect=1:format=rgba,...,lut3d):
    five 4K frames of different brightness with a scene cut at frame 3,
    through the captured chain's params (per-frame detected, temporally
    smoothed peak), against the oracle's sequential model
    (oracle.process_dynamic).  The frames carry MaxCLL 4000 so that the
    detected peak moves instead of sitting at the 1000-nit default cap."""
    import json
    import os
    import numpy as np
    import oracle
    from test_gpu_parity import lattice
    from test_peak_detect import sequence
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'filter_chains.json')
    with open(golden) as fh:
        chain = json.load(fh)['C3']['filter_complex']
    params, _ = hdr2sdr.parse_filter_chain(chain, bits_out=10, maxcll=4000.0)
    assert params.peak_detect and params.resolved_pipeline() == 'libplacebo' and params.lp_p010 == 'truncate'
    W, H = 3840, 2160
    buf = sequence(W, H)[:5]
    t = hdr2sdr.Tonemapper(0, params, lattice(65))
    src = hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 10)
    dst = hdr2sdr.FrameBatch.empty_numpy(5, W, H, 10)
    t.process(src, dst)
    state = t.peak_state()
    t.close()
    knees = []
    want, peaks = oracle.process_dynamic(oracle.params_from(params.to_c()), lattice(65), buf, W, H, knees=knees)
    assert len(set(round(p, 3) for p in peaks)) >= 2, peaks        # the peak really moves
    assert state['frames'] == 5 and state['peak'] == pytest.approx(peaks[-1], rel=1e-4)
    assert_close_int(params, dst.buf.astype(np.int64), want.astype(np.int64), W, H, buf, knees=knees)


def _lp_exact_bound(params, got, want, W, H):
    """H2S_OPT_LP_EXACT: every output sample within one step of the oracle's
    (no k8 lattice-flip allowance, no share beyond)."""
    import numpy as np
    import oracle
    from test_gpu_parity import parity_report
    op = oracle.params_from(params.to_c())
    q = oracle.quant_bits(op)
    step = 1 << max(0, params.bits_out - q)
    parity_report(params, got, want, W, H, q)
    d = np.abs(got - want)
    assert d.max(initial=0) <= step, f'max diff {d.max()} > one step ({step}); {(d > step).sum()} samples beyond'


@pytest.mark.parametrize('kind', ['smooth', 'website'])
def test_c3_lp_exact_full_size_within_one_step(kind):
    """C3 (4K BT.2390, libplacebo branch, 65^3) with H2S_OPT_LP_EXACT on a
    smooth synthetic frame and the reference's own website frame: max diff
    one output step."""
    import os
    import numpy as np
    import oracle
    from hdr2sdr import _abi
    from hdr2sdr.synth import synth_frames, frames_from_rgb8
    from test_gpu_parity import lattice
    W, H = 3840, 2160
    params = hdr2sdr.TonemapParams(tonemapper='bt.2390', gamma=1.0, bits_out=10)
    if kind == 'website':
        z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'website_hdr_full.npz'))
        src = frames_from_rgb8(z[z.files[0]], 1, 10)
    else:
        src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=11)
    t = hdr2sdr.Tonemapper(0, params, lattice(65))
    t.set_option(_abi.OPT_LP_EXACT, 1)
    got = t(src.to_torch('cuda')).to_numpy().buf.astype(np.int64)
    t.close()
    want = oracle.process(oracle.params_from(params.to_c()), lattice(65), src.to_numpy().buf, W, H).astype(np.int64)
    _lp_exact_bound(params, got, want, W, H)


def test_c3_lp_exact_4k_sequence_within_one_step():
    """The 5-frame C3 peak_detect sequence above, with H2S_OPT_LP_EXACT: max
    diff one output step on every frame."""
    import json
    import os
    import numpy as np
    import oracle
    from hdr2sdr import _abi
    from test_gpu_parity import lattice
    from test_peak_detect import sequence
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'filter_chains.json')
    with open(golden) as fh:
        chain = json.load(fh)['C3']['filter_complex']
    params, _ = hdr2sdr.parse_filter_chain(chain, bits_out=10, maxcll=4000.0)
    W, H = 3840, 2160
    buf = sequence(W, H)[:5]
    t = hdr2sdr.Tonemapper(0, params, lattice(65))
    t.set_option(_abi.OPT_LP_EXACT, 1)
    src = hdr2sdr.FrameBatch(np.ascontiguousarray(buf), W, H, 10)
    dst = hdr2sdr.FrameBatch.empty_numpy(5, W, H, 10)
    t.process(src, dst)
    t.close()
    want, _ = oracle.process_dynamic(oracle.params_from(params.to_c()), lattice(65), buf, W, H)
    _lp_exact_bound(params, dst.buf.astype(np.int64), want.astype(np.int64), W, H)
