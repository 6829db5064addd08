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


@pytest.mark.gpu
def test_device_libm_matches_libm(libm):
    """the device forms themselves (h2s::libm_powf / libm_expf,
    through the private entry h2stest_libm) equal libm bit for bit on the
    chain's exponents and random inputs, not only their Python emulation."""
    import ctypes as C
    from hdr2sdr import _abi
    L = C.CDLL(_abi.LIB_PATH)
    L.h2stest_libm.restype = C.c_int
    L.h2stest_libm.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    rng = np.random.default_rng(5)
    ys = [f32(1 / PQ_M2), f32(1 / PQ_M1), PQ_M1, PQ_M2, f32(1 / 2.4), 2.4, 0.2, 1.5]
    xs = np.concatenate([rng.uniform(0, 1, 3000), rng.uniform(1, 60, 500), 10.0 ** rng.uniform(-44, 0, 500),
                         [0.0, 1.0, 1e-45, 1.1754944e-38, 0.5, 0.8359375, 1e6, 0.42890801418277075]]).astype(np.float32)
    for y in ys:
        yv = np.full(xs.shape, y, np.float32)
        out = np.empty_like(xs)
        assert L.h2stest_libm(0, xs.ctypes.data, yv.ctypes.data, out.ctypes.data, xs.size) == 0
        want = np.array([libm.powf(float(x), y) for x in xs], np.float32)
        bad = np.nonzero(out.view(np.uint32) != want.view(np.uint32))[0]
        assert bad.size == 0, [(float(xs[i]), y, float(out[i]), float(want[i])) for i in bad[:5]]
    ex = np.concatenate([rng.uniform(-0.4, 2.6, 3000), rng.uniform(-104, 89, 1000)]).astype(np.float32)
    out = np.empty_like(ex)
    assert L.h2stest_libm(1, ex.ctypes.data, None, out.ctypes.data, ex.size) == 0
    want = np.array([libm.expf(float(x)) for x in ex], np.float32)
    bad = np.nonzero(out.view(np.uint32) != want.view(np.uint32))[0]
    assert bad.size == 0, [(float(ex[i]), float(out[i]), float(want[i])) for i in bad[:5]]
