"""GPU: the host-buffer pipeline (h2s_process cuts a host batch into chunks:
H2D | kernel | D2H on three streams) against the device-resident path, for
the chains and switches whose launches are not a single tile-kernel pass:
the libplacebo branch, BICUBIC chroma (one two-pass launch pair per frame,
one context scratch), dynamic peak detection (per-frame statistics, the IIR
in frame order across chunks), 12-bit HLG with bit replication; at a ragged
size (tile kernel + generic tail) and an odd frame count.  The device path is
also held to the oracle (src/conversion.py:209-224 streams frames through
the same chain)."""
import numpy as np
import pytest

import hdr2sdr
from hdr2sdr.synth import synth_frames

from test_gpu_parity import assert_close_int, lattice
import oracle

pytestmark = pytest.mark.gpu

CASES = {
    'lp_bt2390': dict(tonemapper='bt.2390'),
    'lp_bt2390_peak_detect': dict(tonemapper='bt.2390', peak_detect=True, maxcll=4000.0),
    'cpu_bicubic': dict(tonemapper='hable', gamma=2.2, chroma_filter='bicubic'),
    'cpu_hlg12_replicate_dither': dict(tonemapper='hable', transfer='arib-std-b67', bits_in=12, bits_out=12,
                                       expand='replicate', dither='ordered'),
    'lp_spline_8bit_bicubic': dict(tonemapper='spline', bits_out=8, chroma_filter='bicubic'),
    # dynamic peak with the per-frame two-pass chroma, and with both dithers
    'lp_bt2390_peak_detect_bicubic': dict(tonemapper='bt.2390', peak_detect=True, maxcll=4000.0,
                                          chroma_filter='bicubic'),
    'lp_spline_peak_detect_dithers_eq': dict(tonemapper='spline', peak_detect=True, maxcll=4000.0, gamma=1.3,
                                             dither='ordered', lp_dither='ordered'),
}
F, W, H = 7, 200, 70   # uneven chunks; 3 whole tiles + an 8-pixel generic tail per row; 16-byte rows


@pytest.fixture(scope='module')
def tm():
    t = hdr2sdr.Tonemapper(0)
    yield t
    t.close()


def _run(tm, params, src_in, dst):
    import torch
    if params.peak_detect:
        tm.reset_peak()
    tm.process(src_in, dst)
    torch.cuda.synchronize()
    return dst.to_numpy().buf.astype(np.int64)


@pytest.mark.parametrize('where', ['host_host', 'host_dev', 'dev_host'])
@pytest.mark.parametrize('case', sorted(CASES))
def test_host_pipeline_equals_device_path(tm, case, where):
    params = hdr2sdr.TonemapParams(**CASES[case])
    tm.set_params(params)
    tm.set_lut(lattice(65))
    src = synth_frames('smooth', F, W, H, params.bits_in, device='cpu', seed=17)
    want = _run(tm, params, src.to_torch('cuda'), hdr2sdr.FrameBatch.empty_torch(F, W, H, params.bits_out, 'cuda'))
    src_in = src.to_numpy() if where.startswith('host') else src.to_torch('cuda')
    dst = (hdr2sdr.FrameBatch.empty_pinned(F, W, H, params.bits_out) if where.endswith('host')
           else hdr2sdr.FrameBatch.empty_torch(F, W, H, params.bits_out, 'cuda'))
    got = _run(tm, params, src_in, dst)
    assert np.array_equal(got, want)
    if not params.peak_detect:   # (the dynamic peak's oracle flow is tests/test_peak_detect.py's)
        ref = oracle.process(oracle.params_from(params.to_c()), lattice(65), src.to_numpy().buf, W, H).astype(np.int64)
        assert_close_int(params, want, ref, W, H, src.to_numpy().buf)
