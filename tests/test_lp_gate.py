"""CPU tests of the libplacebo branch's integer gate (tests/lp_gate.py,
VERDICT r05 item 1) and of the oracle's exact stage 1-3 form it judges
against (oracle/h2s_oracle.c chain_lp_d).

* The oracle's own round-5 float32 form of the branch (oracle.lp_form(f32))
  is a float32 implementation like any other: every output sample it puts
  beyond one step from the exact form must be attributed to a download
  channel within the float32 bound of a rounding tie.
* A one-code stage-3 bias (every rgba8 download code + 1 or - 1) must be
  rejected: most of the samples it moves have no channel near a tie.
* The exact form against itself: nothing beyond one step.
"""
import numpy as np
import pytest

import hdr2sdr
import lp_gate
import oracle
from float_gate import lattice
from hdr2sdr.synth import synth_frames

CASES = {
    'C3_bt2390': dict(tonemapper='bt.2390', bits_out=10),
    'C3_max_rgb': dict(tonemapper='bt.2390', bits_out=10, lp_tone='max-rgb'),
    'spline_hlg12': dict(tonemapper='spline', bits_in=12, bits_out=12, transfer='arib-std-b67'),
    'hable_lp': dict(tonemapper='hable', bits_out=10, pipeline='libplacebo'),
    'C3_gamma13': dict(tonemapper='bt.2390', bits_out=10, gamma=1.3),
    'C3_limited_dither': dict(tonemapper='bt.2390', bits_out=10, lp_range='limited', lp_dither='ordered'),
    'C3_bicubic': dict(tonemapper='bt.2390', bits_out=10, chroma_filter='bicubic'),
}
W, H = 256, 128


def _run(kw, kind, **form):
    p = hdr2sdr.TonemapParams(**kw)
    op = oracle.params_from(p.to_c())
    src = synth_frames(kind, 2, W, H, p.bits_in, device='cpu', seed=5).to_numpy().buf
    want = oracle.process(op, lattice(65), src, W, H).astype(np.int64)
    with oracle.lp_form(**form):
        got = oracle.process(op, lattice(65), src, W, H).astype(np.int64)
    return p, src, got, want


@pytest.mark.parametrize('kind', ['smooth', 'uniform', 'ramp', 'edges'])
@pytest.mark.parametrize('case', sorted(CASES))
def test_float32_form_flips_are_attributed(case, kind):
    p, src, got, want = _run(CASES[case], kind, f32=True)
    rep, fails = lp_gate.check(p, 'generic', got, want, src, W, H)
    assert not fails, (rep, fails)


@pytest.mark.parametrize('bias', [1, -1])
@pytest.mark.parametrize('case', ['C3_bt2390', 'spline_hlg12', 'C3_bicubic', 'C3_gamma13'])
def test_one_code_stage3_bias_is_rejected(case, bias):
    p, src, got, want = _run(CASES[case], 'smooth', bias=bias)
    rep, fails = lp_gate.check(p, 'k_tile', got, want, src, W, H)
    assert rep['unattributed'] > 0 and fails, rep
    # most of the moved samples sit nowhere near a tie (a bicubic chroma
    # sample reads 56 pixels, so most of its samples have one near a tie:
    # the luma samples carry the rejection there)
    assert rep['unattributed'] > (0.2 if case == 'C3_bicubic' else 0.8) * rep['beyond'], rep


@pytest.mark.parametrize('case', sorted(CASES))
def test_exact_form_is_its_own_fixed_point(case):
    p, src, got, want = _run(CASES[case], 'uniform')
    assert np.array_equal(got, want)
    rep, fails = lp_gate.check(p, 'exact', got, want, src, W, H)
    assert rep['beyond'] == 0 and not fails


def test_download_values_round_to_the_oracle_codes():
    """oracle.lp_download's x: floor(x) is the download code the chain used
    (checked through stage 4 with the LUT's identity corners: lut3d's 8-bit
    output of an exact lattice node is the node)."""
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
    op = oracle.params_from(p.to_c())
    src = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=2).to_numpy().buf
    x = oracle.lp_download(op, lattice(65), src, W, H)
    s3 = oracle.debug_float(op, lattice(65), src, W, H, 3).astype(np.float64)
    assert np.all(np.abs(np.clip(s3, 0, 1) * 255 + 0.5 - x) < 1e-4)
    assert np.isfinite(x).all()


def test_oracle_lut8x_table_is_lut3d_8bit():
    """oracle.lut8x_table (the reference the GPU suite compares the tile
    kernel's whole table with): the lattice nodes come back truncated to 8
    bits where the code lands exactly on a node (q = 0 and q = 255), and the
    table agrees with the oracle chain's own lut3d stage (the stage-4 plane of
    the debug output) on a frame's download codes."""
    lat = lattice(65)
    tab = oracle.lut8x_table(lat)
    l = np.asarray(lat, np.float32).reshape(-1, 3)
    for code, node in ((0, 0), (255, 65 ** 3 - 1)):
        want = np.minimum(np.maximum((l[node] * np.float32(255.0)).astype(np.int64), 0), 255)
        got = int(tab[code | code << 8 | code << 16])
        assert [got & 255, (got >> 8) & 255, got >> 16] == list(want)
    p = hdr2sdr.TonemapParams(tonemapper='bt.2390', bits_out=10)
    op = oracle.params_from(p.to_c())
    src = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=3).to_numpy().buf
    q = np.floor(oracle.lp_download(op, lat, src, W, H)).astype(np.int64)        # [3, H, W] rgba8 codes
    s4 = oracle.debug_float(op, lat, src, W, H, 4).astype(np.float64)           # lut3d's 8-bit output / 255
    e = tab[(q[0] | q[1] << 8 | q[2] << 16).ravel()]
    got = np.stack([e & 255, (e >> 8) & 255, e >> 16]).reshape(3, H, W).astype(np.float64)
    assert np.array_equal(got, np.rint(s4.reshape(3, H, W) * 255.0))
