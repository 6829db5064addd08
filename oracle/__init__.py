"""Oracle — CPU restatement of the reference's hot path.

TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package, and only as the checker / CPU
baseline.  The product (hdr-to-sdr_amd/hdr2sdr + libh2s) never imports, links
or executes anything here.

Contents
* h2s_oracle.c (built to build/liboracle.so) — the per-pixel chain of
  src/utils.py:38-42 restated stage by stage from the upstream algorithms
  (zimg, vf_tonemap, vf_lut3d, vf_eq, swscale), see that file's header.
* generate_cube_lines / convert — pure-Python restatement of
  tools/generate_lut.py:36-109 (pinned: byte-identical to the reference's own
  generator, sha256 in tests/golden/lut_hashes.json).
* parse_cube — .cube text -> float32 the way lut3d reads it.

Parity status: the LUT lattice is pinned exactly against the reference's
generator.  The pixel stages S1-S8 live in ffmpeg N-125146-gc6bb22dea0 + zimg,
which is absent from this container and not vendored: those stages are
restatements of the published algorithms, pinned only by the reference's
tests that do not need ffmpeg (argv goldens, LUT drift) — pixel parity against
the real ffmpeg binary is UNPINNED (DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'build', 'liboracle.so')


class Params(ctypes.Structure):
    """Layout of h2s_params (include/h2s.h)."""
    _fields_ = [
        ('transfer_in', ctypes.c_int32), ('bits_in', ctypes.c_int32),
        ('bits_out', ctypes.c_int32), ('tonemap', ctypes.c_int32),
        ('tm_param', ctypes.c_double), ('desat', ctypes.c_double),
        ('peak', ctypes.c_double), ('npl', ctypes.c_double),
        ('gamma', ctypes.c_double), ('maxcll', ctypes.c_double),
        ('mastering_max', ctypes.c_double), ('lut_enabled', ctypes.c_int32),
        ('mode', ctypes.c_int32), ('desat_luma', ctypes.c_int32),
        ('peak_detect', ctypes.c_int32),
        ('chroma_filter', ctypes.c_int32), ('dither', ctypes.c_int32),
        ('expand', ctypes.c_int32), ('pipeline', ctypes.c_int32),
        ('knee_offset', ctypes.c_double), ('target_black', ctypes.c_double),
        ('target_white', ctypes.c_double),
        ('chroma_edge', ctypes.c_int32),
        ('lut_input', ctypes.c_int32),
        ('lp_tone', ctypes.c_int32),
        # ABI v3: libplacebo branch options and peak_detect parameters
        ('lp_range', ctypes.c_int32), ('lp_dither', ctypes.c_int32), ('lp_p010', ctypes.c_int32),
        ('reserved', ctypes.c_int32 * 2),
        ('pd_smoothing', ctypes.c_double), ('pd_scene_low', ctypes.c_double),
        ('pd_scene_high', ctypes.c_double), ('pd_percentile', ctypes.c_double),
        ('pd_min_peak', ctypes.c_double),
    ]


class Frames(ctypes.Structure):
    """Layout of h2s_frames (include/h2s.h)."""
    _fields_ = [
        ('data', ctypes.c_void_p * 3), ('linesize', ctypes.c_int64 * 3),
        ('frame_pitch', ctypes.c_int64 * 3), ('width', ctypes.c_int32),
        ('height', ctypes.c_int32), ('bits', ctypes.c_int32),
        ('location', ctypes.c_int32),
    ]


def params_from(obj) -> Params:
    """Copy same-named fields from any h2s_params-like object."""
    p = Params()
    for name, _ in Params._fields_:
        if name == 'reserved':
            continue
        setattr(p, name, getattr(obj, name))
    return p


def default_params(**kw) -> Params:
    """Reference chain defaults (see include/h2s.h h2s_params_default)."""
    p = Params(transfer_in=0, bits_in=10, bits_out=10, tonemap=6, tm_param=math.nan,
               desat=2.0, peak=0.0, npl=100.0, gamma=1.0, maxcll=0.0, mastering_max=0.0,
               lut_enabled=1, mode=0, desat_luma=0, knee_offset=math.nan, target_black=math.nan,
               target_white=math.nan)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f'{LIB_PATH} missing: run __graft_entry__.build()')
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_process.restype = ctypes.c_int
        L.oracle_process.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int,
                                     ctypes.POINTER(Frames), ctypes.POINTER(Frames), ctypes.c_int,
                                     ctypes.c_int]
        L.oracle_process_knee.restype = ctypes.c_int
        L.oracle_process_knee.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int,
                                          ctypes.POINTER(Frames), ctypes.POINTER(Frames), ctypes.c_int,
                                          ctypes.c_int, ctypes.c_double]
        L.oracle_debug_float_knee.restype = ctypes.c_int
        L.oracle_debug_float_knee.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int,
                                              ctypes.POINTER(Frames), ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
        L.oracle_tonemap_lin_knee.restype = ctypes.c_int
        L.oracle_tonemap_lin_knee.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
        L.oracle_debug_float.restype = ctypes.c_int
        L.oracle_debug_float.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int,
                                         ctypes.POINTER(Frames), ctypes.c_int, ctypes.c_void_p]
        L.oracle_resolved.restype = ctypes.c_int
        L.oracle_resolved.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double), ctypes.c_void_p, ctypes.c_int]
        L.oracle_tone_curve.restype = ctypes.c_float
        L.oracle_tone_curve.argtypes = [ctypes.POINTER(Params), ctypes.c_float]
        L.oracle_pq_eotf.restype = ctypes.c_float
        L.oracle_pq_eotf.argtypes = [ctypes.c_float]
        L.oracle_hlg_inverse_oetf.restype = ctypes.c_float
        L.oracle_hlg_inverse_oetf.argtypes = [ctypes.c_float]
        L.oracle_peak_stats.restype = ctypes.c_int
        L.oracle_peak_stats.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(Frames), ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_chroma_taps.restype = None
        L.oracle_chroma_taps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_tonemap_lin.restype = ctypes.c_int
        L.oracle_tonemap_lin.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_void_p]
        L.oracle_set_lp_f32.restype = None
        L.oracle_set_lp_f32.argtypes = [ctypes.c_int]
        L.oracle_set_lp_bias.restype = None
        L.oracle_set_lp_bias.argtypes = [ctypes.c_int]
        L.oracle_lp_download.restype = ctypes.c_int
        L.oracle_lp_download.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_int,
                                         ctypes.POINTER(Frames), ctypes.c_double, ctypes.c_void_p]
        L.oracle_preview_tail.restype = ctypes.c_int
        L.oracle_preview_tail.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
        _lib = L
    return _lib


def _frames(buf: np.ndarray, width: int, height: int, bits: int) -> Frames:
    """Descriptor for a contiguous [F, W*H*3/2] host batch (hdr2sdr layout)."""
    assert buf.flags['C_CONTIGUOUS']
    sb = 1 if bits == 8 else 2
    ysz = width * height * sb
    csz = ysz // 4
    d = Frames()
    base = buf.ctypes.data
    d.data[0], d.data[1], d.data[2] = base, base + ysz, base + ysz + csz
    d.linesize[0] = width * sb
    d.linesize[1] = d.linesize[2] = width // 2 * sb
    for p in range(3):
        d.frame_pitch[p] = ysz + 2 * csz
    d.width, d.height, d.bits, d.location = width, height, bits, 1
    return d


def process(params: Params, lattice: 'np.ndarray | None', buf: np.ndarray, width: int, height: int,
            nthreads: int = 0, avg_pq: float = 0.0) -> np.ndarray:
    """Run the restated chain over a host batch; returns the output batch
    (uint8 for bits_out 8, else uint16).  avg_pq > 0 sets the spline knee's
    source level (peak detection)."""
    bits_in, bits_out = params.bits_in, params.bits_out
    out = np.zeros((buf.shape[0], width * height * 3 // 2), dtype=np.uint8 if bits_out == 8 else np.uint16)
    din = _frames(np.ascontiguousarray(buf), width, height, bits_in)
    dout = _frames(out, width, height, bits_out)
    lat, n = (None, 0)
    if lattice is not None:
        lat = np.ascontiguousarray(lattice, dtype=np.float32).reshape(-1, 3)
        n = round(lat.shape[0] ** (1 / 3))
    rc = lib().oracle_process_knee(ctypes.byref(params), lat.ctypes.data if lat is not None else None, n,
                                   ctypes.byref(din), ctypes.byref(dout), buf.shape[0], nthreads, avg_pq)
    if rc:
        raise ValueError(f'oracle_process failed: {rc}')
    return out


def debug_float(params: Params, lattice: 'np.ndarray | None', buf: np.ndarray, width: int, height: int,
                stage: int, avg_pq: float = 0.0) -> np.ndarray:
    out = np.empty((3, height, width), dtype=np.float32)
    din = _frames(np.ascontiguousarray(buf[:1]), width, height, params.bits_in)
    lat, n = (None, 0)
    if lattice is not None:
        lat = np.ascontiguousarray(lattice, dtype=np.float32).reshape(-1, 3)
        n = round(lat.shape[0] ** (1 / 3))
    rc = lib().oracle_debug_float_knee(ctypes.byref(params), lat.ctypes.data if lat is not None else None, n,
                                       ctypes.byref(din), stage, float(avg_pq), out.ctypes.data)
    if rc:
        raise ValueError(f'oracle_debug_float failed: {rc}')
    return out


def tonemap_lin(params: Params, lattice: 'np.ndarray | None', rgb: np.ndarray, avg_pq: float = 0.0) -> np.ndarray:
    """S2 alone (the chain's tone map, oracle tonemap_px) on linear R'G'B'
    planes rgb[3, ...] in units of npl; float32 like the chain."""
    shp = rgb.shape
    a = np.ascontiguousarray(rgb, dtype=np.float32).reshape(3, -1)
    out = np.empty_like(a)
    lat, n = (None, 0)
    if lattice is not None:
        lat = np.ascontiguousarray(lattice, dtype=np.float32).reshape(-1, 3)
        n = round(lat.shape[0] ** (1 / 3))
    rc = lib().oracle_tonemap_lin_knee(ctypes.byref(params), lat.ctypes.data if lat is not None else None, n,
                                       a.ctypes.data, a.shape[1], float(avg_pq), out.ctypes.data)
    if rc:
        raise ValueError(f'oracle_tonemap_lin failed: {rc}')
    return out.reshape(shp)


def lut8x_table(lattice: np.ndarray) -> np.ndarray:
    """lut3d's 8-bit path (oracle lut3d_8bit) for every rgba8 code triple:
    2^24 uint32, R | G << 8 | B << 16 at index r | g << 8 | b << 16."""
    lat = np.ascontiguousarray(lattice, dtype=np.float32).reshape(-1, 3)
    n = round(lat.shape[0] ** (1 / 3))
    out = np.empty(1 << 24, dtype=np.uint32)
    L = lib()
    L.oracle_lut8x_table.restype = ctypes.c_int
    L.oracle_lut8x_table.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    rc = L.oracle_lut8x_table(lat.ctypes.data, n, out.ctypes.data)
    if rc:
        raise ValueError(f'oracle_lut8x_table failed: {rc}')
    return out


def lp_download(params: Params, lattice: np.ndarray, buf: np.ndarray, width: int, height: int,
                avg_pq: float = 0.0) -> np.ndarray:
    """libplacebo branch with the LUT: the exact (double) pre-rounding value x
    of every rgba8 download channel of frame 0, [3, H, W] float64; the code is
    floor(x).  The tie attribution of tests/lp_gate.py reads it."""
    out = np.empty((3, height, width), dtype=np.float64)
    din = _frames(np.ascontiguousarray(buf[:1]), width, height, params.bits_in)
    lat = np.ascontiguousarray(lattice, dtype=np.float32).reshape(-1, 3)
    n = round(lat.shape[0] ** (1 / 3))
    rc = lib().oracle_lp_download(ctypes.byref(params), lat.ctypes.data, n, ctypes.byref(din), float(avg_pq),
                                  out.ctypes.data)
    if rc:
        raise ValueError(f'oracle_lp_download failed: {rc}')
    return out


class lp_form:
    """Context manager: the libplacebo branch's stages 1-3 in the round-5
    float32 form (f32=True) instead of exact arithmetic, and / or a bias of
    `bias` codes on every rgba8 download code (the gate's mutation tests).
    Process-wide; restores the defaults (exact, no bias) on exit."""

    def __init__(self, f32: bool = False, bias: int = 0):
        self.f32, self.bias = f32, bias

    def __enter__(self):
        lib().oracle_set_lp_f32(1 if self.f32 else 0)
        lib().oracle_set_lp_bias(self.bias)
        return self

    def __exit__(self, *exc):
        lib().oracle_set_lp_f32(0)
        lib().oracle_set_lp_bias(0)
        return False


def preview_rgb24(params: Params, lattice: 'np.ndarray | None', buf: np.ndarray, width: int, height: int,
                  out_w: int, out_h: int, gamma: float = 1.0) -> np.ndarray:
    """Preview of frame 0: the chain at bits_out 8 (with peak_detect: the
    frame's own detected peak from a fresh state, as each of the reference's
    preview ffmpeg runs starts one, src/utils.py:768-800), then the restated
    scale / yuv420p->rgb24 / adjust_gamma tail (PARITY UNPINNED, see h2s_oracle.c)."""
    if params.bits_out != 8:
        raise ValueError('preview runs the chain at bits_out 8')
    one = np.ascontiguousarray(buf[:1])
    if params.peak_detect:
        yuv8 = np.ascontiguousarray(process_dynamic(params, lattice, one, width, height)[0][0])
    else:
        yuv8 = np.ascontiguousarray(process(params, lattice, one, width, height)[0])
    out = np.zeros((out_h, out_w, 3), dtype=np.uint8)
    rc = lib().oracle_preview_tail(yuv8.ctypes.data, width, height, out_w, out_h, float(gamma), out.ctypes.data)
    if rc:
        raise ValueError(f'oracle_preview_tail failed: {rc}')
    return out


def peak_stats(params: Params, buf: np.ndarray, width: int, height: int) -> 'tuple[np.ndarray, np.ndarray]':
    """Per-frame (max, mean) of the PQ-encoded max(R,G,B) (PARITY UNPINNED)."""
    n = buf.shape[0]
    fmax, favg = np.zeros(n), np.zeros(n)
    d = _frames(np.ascontiguousarray(buf), width, height, params.bits_in)
    rc = lib().oracle_peak_stats(ctypes.byref(params), ctypes.byref(d), n, fmax.ctypes.data, favg.ctypes.data)
    if rc:
        raise ValueError(f'oracle_peak_stats failed: {rc}')
    return fmax, favg


def pq_eotf_d(e: float) -> float:
    """ST 2084 EOTF in double, 1.0 = 10000 nits."""
    m1, m2 = 2610 / 16384, 2523 / 4096 * 128
    c1, c2, c3 = 3424 / 4096, 2413 / 4096 * 32, 2392 / 4096 * 32
    if not e > 0:
        return 0.0
    xp = e ** (1 / m2)
    return (max(xp - c1, 0.0) / (c2 - c3 * xp)) ** (1 / m1)


def _nan_or(v, d):
    return d if v is None or (isinstance(v, float) and math.isnan(v)) else v


class PeakState:
    """Restatement of the dynamic-peak smoothing (h2s_api.hip peak_update;
    PARITY UNPINNED): IIR with coefficient 1 - exp(-1 / smoothing_period) on
    the PQ peak measurement / average, bypassed by a smoothstep over the
    scene-change band (% PQ average change); the peak clamped to
    [minimum_peak x SDR white, static].  Defaults: vf_libplacebo's options
    (100 frames, 5.5 / 10 %, minimum_peak 1.0) for ``params`` with NaN
    fields; ``params`` None keeps those defaults with a 203-nit white."""

    def __init__(self, params=None, **kw):
        self.frames, self.max, self.avg = 0, 0.0, 0.0

        def g(n, d):
            if n in kw:
                return kw[n]
            return _nan_or(getattr(params, n, None), d) if params is not None else d
        self.smoothing = g('pd_smoothing', 100.0)
        self.lo, self.hi = g('pd_scene_low', 5.5), g('pd_scene_high', 10.0)
        white = 203.0
        if params is not None:
            lp = params.pipeline == 2 or (params.pipeline == 0 and params.tonemap in (7, 8))
            white = _nan_or(params.target_white, 203.0 if lp else params.npl)
        white = kw.get('white', white)
        self.min_peak = g('pd_min_peak', 1.0) * white / 100.0

    def update(self, fmax: float, favg: float, static_peak: float) -> float:
        if self.frames == 0:
            self.max, self.avg = fmax, favg
        else:
            a = 1.0 - math.exp(-1.0 / self.smoothing) if self.smoothing > 0 else 1.0
            d = abs(favg - self.avg) * 100.0
            t = 0.0
            if self.lo >= 0 and self.hi >= 0:
                t = (d - self.lo) / (self.hi - self.lo) if self.hi > self.lo else (1.0 if d >= self.lo else 0.0)
            t = min(max(t, 0.0), 1.0)
            w = a + (1.0 - a) * t * t * (3.0 - 2.0 * t)
            self.max += w * (fmax - self.max)
            self.avg += w * (favg - self.avg)
        self.frames += 1
        return min(max(pq_eotf_d(self.max) * 100.0, self.min_peak), static_peak)


def process_dynamic(params: Params, lattice: 'np.ndarray | None', buf: np.ndarray, width: int, height: int,
                    state: 'PeakState | None' = None, knees: 'list | None' = None) -> 'tuple[np.ndarray, list[float]]':
    """BT.2390 / spline with the detected peak: stats, smoothing, then each
    frame through the chain with its own peak (and, for spline, the smoothed
    average as the knee source).  Returns (frames, peaks); knees (a list, if
    given) receives each frame's (peak, average PQ) -- the static parameters
    a per-frame check of that frame needs (tests/lp_gate.py)."""
    state = state or PeakState(params)
    static_peak = resolved(params)[0]
    fmax, favg = peak_stats(params, buf, width, height)
    outs, peaks = [], []
    for f in range(buf.shape[0]):
        pk = state.update(float(fmax[f]), float(favg[f]), static_peak)
        q = params_from(params)
        q.peak = pk
        outs.append(process(q, lattice, np.ascontiguousarray(buf[f:f + 1]), width, height, avg_pq=state.avg))
        peaks.append(pk)
        if knees is not None:
            knees.append((pk, state.avg))
    return np.concatenate(outs), peaks


def resolved(params: Params) -> 'tuple[float, float, np.ndarray]':
    """(peak, param, eq_lut) after vf_tonemap / vf_eq initialisation."""
    peak, param = ctypes.c_double(), ctypes.c_double()
    eq = np.zeros(4096, dtype=np.uint16)
    q = lib().oracle_resolved(ctypes.byref(params), ctypes.byref(peak), ctypes.byref(param),
                              eq.ctypes.data, eq.size)
    if q < 0:
        raise ValueError(f'oracle_resolved failed: {q}')
    return peak.value, param.value, eq[:1 << q].copy()


def quant_bits(params: Params) -> int:
    """The depth the chain quantises at: 8 (eq's yuv420p, or the libplacebo
    branch's nv12) or bits_out (native mode; libplacebo rgba with gamma 1)."""
    q = lib().oracle_resolved(ctypes.byref(params), None, None, None, 0)
    if q < 0:
        raise ValueError(f'oracle_resolved failed: {q}')
    return q


def chroma_taps() -> 'tuple[np.ndarray, np.ndarray]':
    """The BICUBIC chroma decimation taps (7 horizontal, 8 vertical)."""
    wx, wy = np.zeros(7, np.float32), np.zeros(8, np.float32)
    lib().oracle_chroma_taps(wx.ctypes.data, wy.ctypes.data)
    return wx, wy


def tone_curve(params: Params, sig: float) -> float:
    return float(lib().oracle_tone_curve(ctypes.byref(params), sig))


def pq_eotf(x: float) -> float:
    return float(lib().oracle_pq_eotf(x))


def hlg_inverse_oetf(x: float) -> float:
    return float(lib().oracle_hlg_inverse_oetf(x))


# ---- tools/generate_lut.py restated (pure Python) --------------------------
BT2020_TO_BT709 = [  # tools/generate_lut.py:36-40
    [1.6604910021, -0.5876411388, -0.0728498633],
    [-0.1245504745, 1.1328998971, -0.0083494226],
    [-0.0181507634, -0.1005788980, 1.1187296614],
]


def convert(r: float, g: float, b: float) -> 'tuple[float, float, float]':
    """tools/generate_lut.py:75-90: 2.4 decode, matrix, clamp, 1/2.4 encode."""
    lin = [r ** 2.4, g ** 2.4, b ** 2.4]                         # :43-59
    m = BT2020_TO_BT709
    out = []
    for row in m:
        v = row[0] * lin[0] + row[1] * lin[1] + row[2] * lin[2]
        v = max(0.0, min(1.0, v))                                # :71-72
        out.append(v ** (1 / 2.4))                               # :62-68
    return out[0], out[1], out[2]


def generate_cube_lines(size: int) -> 'list[str]':
    """tools/generate_lut.py:93-109: header + size^3 lines, red fastest."""
    lines = [f'LUT_3D_SIZE {size}']
    for bi in range(size):
        b = bi / (size - 1)
        for gi in range(size):
            g = gi / (size - 1)
            for ri in range(size):
                r = ri / (size - 1)
                o = convert(r, g, b)
                lines.append(f'{o[0]:.6f} {o[1]:.6f} {o[2]:.6f}')
    return lines


def parse_cube(text: str) -> np.ndarray:
    """lut3d's .cube read: data lines -> float32 [n^3, 3] (decimal -> double
    -> float, as av_strtod + cast)."""
    n = None
    vals = []
    for line in text.splitlines():
        s = line.strip()
        if not s or s.startswith('#') or s.startswith('TITLE') or s.startswith('DOMAIN_'):
            continue
        if s.startswith('LUT_3D_SIZE'):
            n = int(s.split()[1])
            continue
        vals.append([float(t) for t in s.split()[:3]])
    a = np.asarray(vals, dtype=np.float64).astype(np.float32)
    assert n is not None and a.shape == (n ** 3, 3), (n, a.shape)
    return a
