"""The generic kernel's powf / expf tables (hdr-to-sdr_amd/csrc/h2s_libm.h)
are the ones of the libm the oracle links: a pure-Python evaluation of
glibc's forms over the committed tables (tests/libm_emu.py, the device
h2s::libm_powf / libm_expf written out) equals libm.powf / libm.expf bit for
bit on the exponents the chain uses and on random ones.  A different libm
under the oracle fails here first (regenerate with scripts/
gen_libm_tables.py).  CPU only."""
import ctypes
import ctypes.util
import os

import numpy as np
import pytest

from libm_emu import emu_expf, emu_powf, parse_header

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'hdr-to-sdr_amd', 'csrc', 'h2s_libm.h')


@pytest.fixture(scope='module')
def libm():
    L = ctypes.CDLL(ctypes.util.find_library('m'))
    L.powf.restype = ctypes.c_float
    L.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    L.expf.restype = ctypes.c_float
    L.expf.argtypes = [ctypes.c_float]
    return L


@pytest.fixture(scope='module')
def tables():
    T = parse_header(HDR)
    assert len(T.log2_tab) == 16 and len(T.log2_poly) == 5 and len(T.exp2_tab) == 32
    assert len(T.exp2_poly) == 3 and len(T.exp2_poly_scaled) == 3
    return T


def f32(v):
    return float(np.float32(v))


# the chain's exponents: PQ 1/m2, 1/m1, m1, m2; the BT.1886 encode 1/2.4 and
# 2.4; HLG's system gamma 0.2; Hable-free powers of the spline / BT.2390 knee
PQ_M1, PQ_M2 = 0.1593017578125, 78.84375


@pytest.mark.parametrize('y', [f32(1 / PQ_M2), f32(1 / PQ_M1), PQ_M1, PQ_M2, f32(1 / 2.4), 2.4, 0.2, 1.5, f32(1 / 3)])
def test_powf_matches_libm(libm, tables, y):
    rng = np.random.default_rng(int(y * 1000))
    xs = np.concatenate([rng.uniform(0, 1, 1500), rng.uniform(1, 60, 300), 10.0 ** rng.uniform(-44, 0, 400),
                         [0.0, 1.0, 1e-45, 1.1754944e-38, 0.5, 0.8359375, 1e6]])
    bad = [(float(x), emu_powf(tables, f32(x), y), libm.powf(f32(x), y)) for x in xs
           if emu_powf(tables, f32(x), y) != libm.powf(f32(x), y)]
    assert not bad, bad[:5]


def test_expf_matches_libm(libm, tables):
    rng = np.random.default_rng(9)
    xs = np.concatenate([rng.uniform(-0.4, 2.6, 2000), rng.uniform(-104, 89, 1000), [0.0, -0.0, 88.7, -103.9]])
    bad = [(float(x), emu_expf(tables, f32(x)), libm.expf(f32(x))) for x in xs
           if emu_expf(tables, f32(x)) != libm.expf(f32(x))]
    assert not bad, bad[:5]


def test_glibc_powf_is_not_the_correctly_rounded_one(libm, tables):
    """Why the tables: the input of the round-5 C3 flip (pixel 1580, 845),
    E' = 0.42890802f, where libm's x^(1/m2) is one ulp below the correctly
    rounded value (the emulation follows libm, the double form does not)."""
    x, y = f32(0.42890801418277075), f32(1 / PQ_M2)
    cr = f32(float(np.float64(x) ** np.float64(y)))
    assert libm.powf(x, y) == emu_powf(tables, x, y) != cr
