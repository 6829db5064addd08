"""Pure-Python restatement of glibc 2.35's powf / expf (x86-64 FMA variants)
over their constant tables, for scripts/gen_libm_tables.py and
tests/test_libm_tables.py.  The device forms are h2s::libm_powf /
h2s::libm_expf in hdr-to-sdr_amd/csrc/h2s_device.h; this file checks the
tables and the evaluation order against the libm the oracle links.

powf (e_powf.c): log2(x) = k + log2(c) + poly(z / c - 1) from a 16-entry
table indexed by the top mantissa bits (OFF 0x3f330000), y log2(x) in double,
then exp2 as 2^(k/32) (table) x a cubic in the remainder; one rounding to
float at the end.  expf (e_expf.c): the same exp2 tail on x / ln 2.  The
multiply-adds are fused (the FMA build), written fma() here."""
import math
import re
import struct
from dataclasses import dataclass
from fractions import Fraction

import numpy as np


@dataclass
class LibmTables:
    log2_tab: list
    log2_poly: list
    exp2_tab: list
    shift_scaled: float
    exp2_poly: list
    shift: float
    invln2_scaled: float
    exp2_poly_scaled: list


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _asu32(f):
    return struct.unpack('<I', struct.pack('<f', f))[0]


def _asf32(u):
    return struct.unpack('<f', struct.pack('<I', u & 0xffffffff))[0]


def _asu64(d):
    return struct.unpack('<Q', struct.pack('<d', d))[0]


def _asf64(u):
    return struct.unpack('<d', struct.pack('<Q', u & 0xffffffffffffffff))[0]


def _f32(v):
    with np.errstate(over='ignore'):
        return float(np.float32(v))


def _exp2_tail(T, xd, shift, poly):
    kd = xd + shift
    ki = _asu64(kd)
    kd -= shift
    r = xd - kd
    t = (T.exp2_tab[ki % 32] + (ki << 47)) & 0xffffffffffffffff
    s = _asf64(t)
    z = fma(poly[0], r, poly[1])
    r2 = r * r
    y = fma(poly[2], r, 1.0)
    y = fma(z, r2, y)
    return _f32(y * s)


def emu_powf(T, x, y):
    """powf for x >= 0 and finite y != 0 (the oracle's uses)."""
    x, y = _f32(x), _f32(y)
    if math.isnan(x) or math.isnan(y):
        return float('nan')
    if y == 0.0 or x == 1.0:
        return 1.0
    if x < 0.0:
        raise ValueError('negative base is outside the restated range')
    if x == 0.0:
        return 0.0 if y > 0 else float('inf')
    if math.isinf(x):
        return float('inf') if y > 0 else 0.0
    ix = _asu32(x)
    if ix < 0x00800000:                      # subnormal: normalise
        ix = (_asu32(_f32(x * float.fromhex('0x1p23'))) - (23 << 23)) & 0xffffffff
    tmp = (ix - 0x3f330000) & 0xffffffff
    i = (tmp >> 19) % 16
    top = tmp & 0xff800000
    iz = (ix - top) & 0xffffffff
    k = (top - (1 << 32) if top >= 1 << 31 else top) >> 23
    invc, logc = T.log2_tab[i]
    z = _asf32(iz)
    r = fma(z, invc, -1.0)
    y0 = logc + float(k)
    A = T.log2_poly
    r2 = r * r
    yy = fma(A[0], r, A[1])
    p = fma(A[2], r, A[3])
    r4 = r2 * r2
    q = fma(A[4], r, y0)
    q = fma(p, r2, q)
    logx = fma(yy, r4, q)
    ylogx = y * logx
    if ((_asu64(ylogx) >> 47) & 0xffff) >= (_asu64(126.0) >> 47):
        if ylogx > float.fromhex('0x1.fffffffd1d571p+6'):
            return float('inf')
        if ylogx <= -150.0:
            return 0.0
    return _exp2_tail(T, ylogx, T.shift_scaled, T.exp2_poly)


def emu_expf(T, x):
    x = _f32(x)
    if math.isnan(x):
        return x
    if x > float.fromhex('0x1.62e42ep6'):
        return float('inf')
    if x < -float.fromhex('0x1.9fe368p6'):
        return 0.0
    z = T.invln2_scaled * x
    return _exp2_tail(T, z, T.shift, T.exp2_poly_scaled)


def parse_header(path):
    """The tables as h2s_libm.h holds them."""
    txt = open(path).read()

    def block(name):
        m = re.search(name + r'[^{]*=\s*\{(.*?)\};', txt, re.S)
        return m.group(1)

    def nums(s):
        return [float.fromhex(v) if 'p' in v else float(v) for v in re.findall(r'-?0x[0-9a-fA-F.]+p[-+]?\d+|-?0x0\.0p\+0', s)]

    rows = [tuple(float.fromhex(v) for v in pair)
            for pair in re.findall(r'\{(-?0x[0-9a-f.]+p[-+]?\d+), (-?0x[0-9a-f.]+p[-+]?\d+)\}', block('POWF_LOG2_TAB'))]
    exp2 = [int(v, 16) for v in re.findall(r'0x([0-9a-f]{16})ull', block('EXP2F_TAB'))]

    def scalar(name):
        return float.fromhex(re.search(name + r'\s*=\s*(-?0x[0-9a-f.]+p[-+]?\d+);', txt).group(1))
    return LibmTables(log2_tab=rows, log2_poly=nums(block('POWF_LOG2_POLY')), exp2_tab=exp2,
                      shift_scaled=scalar('EXP2F_SHIFT_SCALED'), exp2_poly=nums(block("EXP2F_POLY\\[3\\]")),
                      shift=scalar('EXP2F_SHIFT'), invln2_scaled=scalar('EXP2F_INVLN2_SCALED'),
                      exp2_poly_scaled=nums(block('EXP2F_POLY_SCALED')))
