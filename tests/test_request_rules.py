"""The reference's request -> chain rules, pinned against its own build().

``tests/golden/request_rules.json`` holds the filter graph (or the
``ValueError``) that the reference's ``ffmpeg_command.build()`` produced for a
matrix of ``ConversionRequest`` fields and probe results
(``tests/golden/make_golden.py rules``): use_gpu x operator x bit depth,
lut_enabled x gamma, the CUDA-interop prefix, Dolby Vision profile 5 and an
absent libplacebo.  ``TonemapParams.from_request`` must reproduce every case
(Dolby Vision profile 5 excepted: the drop-in refuses it, see below):

* the same branch (``_tonemap_plan``, src/ffmpeg_command.py:96-144);
* the same params as ``parse_filter_chain`` of the captured string
  (peak_detect=1 and lut_enabled on the libplacebo branch, the p010 upload
  cut for 12-bit input, src/utils.py:392-471);
* the same string back from ``filter_string()``;
* the same ValueError text for bt.2390 / spline on the CPU chain (:240-245).
"""
import json
import os
from dataclasses import dataclass

import pytest

import hdr2sdr
from hdr2sdr import chain as C
from hdr2sdr import preview as PV

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'request_rules.json')
with open(GOLDEN) as _f:
    RULES = json.load(_f)


@dataclass(frozen=True)
class Req:   # src/conversion.py:26-44 (the fields build() reads)
    input_path: str = 'in.mkv'
    output_path: str = 'out.mkv'
    gamma: float = 1.0
    use_gpu: bool = False
    tonemapper: str = 'reinhard'
    quality: int = 23
    quality_mode: str = 'cq'
    bit_depth: int = 10
    licensed: bool = False
    lut_enabled: bool = True


def _case_id(c):
    r = c['req']
    extra = ''.join(f'-{k}' for k in ('encoder', 'props', 'libplacebo') if k in c)
    return (f"{r['tonemapper']}-gpu{int(r['use_gpu'])}-{r['bit_depth']}b-lut{int(r.get('lut_enabled', True))}"
            f"-g{r.get('gamma', 1.0)}{extra}")


def _from_request(c, bits_in=10):
    props = dict(c.get('props', {}))
    interop = c.get('encoder') == 'h264_nvenc' and c.get('interop', False)
    calls = []

    def probe():
        calls.append(1)
        return c.get('libplacebo', True)
    p = hdr2sdr.TonemapParams.from_request(Req(**c['req']), bits_in=bits_in, properties=props,
                                           libplacebo_available=probe, cuda_interop=interop)
    return p, calls


def _dovi5(case):
    return C.is_dovi_profile5(case.get('props'))


@pytest.mark.parametrize('case', RULES['cases'], ids=_case_id)
def test_from_request_reproduces_build(case):
    if _dovi5(case) and 'error' not in case:
        # the reference routes profile 5 to libplacebo for its RPU
        # (src/ffmpeg_command.py:100-106); the drop-in refuses it so that the
        # caller keeps the reference command
        plan = C.tonemap_plan(Req(**case['req']), case['props'], True)
        assert plan.dovi_needs_rpu and plan.use_libplacebo
        assert 'libplacebo=' in case['filter_complex']
        with pytest.raises(ValueError) as e:
            _from_request(case)
        assert str(e.value) == C.DOVI_P5_ERROR
        return
    if 'error' in case:
        with pytest.raises(ValueError) as e:
            _from_request(case)
        assert str(e.value) == case['error']
        return
    p, _ = _from_request(case)
    fc = case['filter_complex']
    # same string back
    assert '[0:v:0]' + p.filter_string() + '[vout]' == fc
    # same params as the parsed string
    pix = {'yuv420p': 8, 'yuv420p10le': 10, 'p010le': 10, 'yuv420p12le': 12}[case['pix_fmt']]
    q, lut = C.parse_filter_chain(fc, bits_out=pix)
    keys = ('tonemapper', 'gamma', 'bits_out', 'lut_enabled', 'peak_detect', 'desat', 'lp_p010', 'npl')
    assert {k: getattr(p, k) for k in keys} == {k: getattr(q, k) for k in keys}
    assert p.resolved_pipeline() == q.resolved_pipeline()
    assert (lut == '<LUT>') == p.lut_enabled


def test_branch_rules_spelled_out():
    """The rules the verdict lists, each on one request."""
    lp = lambda **kw: hdr2sdr.TonemapParams.from_request(Req(**kw))   # noqa: E731
    # use_gpu: every operator through libplacebo, peak detection on
    for tm in ('reinhard', 'mobius', 'hable', 'bt.2390', 'spline'):
        p = lp(tonemapper=tm, use_gpu=True)
        assert p.resolved_pipeline() == 'libplacebo' and p.peak_detect and p.desat == 0.0
    # bit_depth >= 12 forces the CPU chain; the GPU-only operators then raise
    p = lp(tonemapper='hable', use_gpu=True, bit_depth=12)
    assert p.resolved_pipeline() == 'cpu' and p.bits_out == 12 and not p.peak_detect
    with pytest.raises(ValueError, match='requires GPU tonemapping'):
        lp(tonemapper='bt.2390', use_gpu=True, bit_depth=12)
    # lut_enabled honoured on the libplacebo branch, ignored on the CPU chain
    assert not lp(tonemapper='bt.2390', use_gpu=True, lut_enabled=False).lut_enabled
    assert lp(tonemapper='hable', lut_enabled=False).lut_enabled
    # the upload prefix: p010 cuts 12-bit input, the interop hwmap keeps it
    assert lp(tonemapper='bt.2390', use_gpu=True).lp_p010 == 'truncate'
    assert hdr2sdr.TonemapParams.from_request(Req(tonemapper='bt.2390', use_gpu=True),
                                              cuda_interop=True).lp_p010 == 'keep'


def test_libplacebo_probe_is_lazy():
    """src/ffmpeg_command.py:116-119: the probe runs only when use_gpu or
    DoVi profile 5 asks for libplacebo."""
    calls = []

    def probe():
        calls.append(1)
        return True
    hdr2sdr.TonemapParams.from_request(Req(tonemapper='hable'), libplacebo_available=probe)
    hdr2sdr.TonemapParams.from_request(Req(tonemapper='hable', use_gpu=True, bit_depth=12),
                                       libplacebo_available=probe)
    assert calls == []
    hdr2sdr.TonemapParams.from_request(Req(tonemapper='hable', use_gpu=True), libplacebo_available=probe)
    assert calls == [1]


@pytest.mark.parametrize('prefix,want', [('format=p010,hwupload,', 'truncate'), ('hwmap=derive_device=vulkan,', 'keep')])
def test_upload_prefix_sets_p010_model(prefix, want):
    chain = (prefix + 'libplacebo=w=iw:h=ih:tonemapping=bt.2390:colorspace=bt709:color_primaries=auto:'
             'color_trc=bt709:range=tv:peak_detect=1:format=rgba,hwdownload,format=rgba,'
             'lut3d=file=<LUT>:interp=tetrahedral,setparams=color_primaries=bt709:color_trc=bt709:colorspace=bt709')
    p, _ = C.parse_filter_chain(chain, bits_in=12)
    assert p.lp_p010 == want and p.bits_in == 12
    assert p.filter_string() == chain


def test_abi_default_is_the_p010_prefix():
    """h2s_params_default and TonemapParams agree: the reference's default
    upload prefix is format=p010 (src/utils.py:431)."""
    import ctypes
    from hdr2sdr import _abi
    d = _abi.H2SParams()
    _abi.lib().h2s_params_default(ctypes.byref(d))
    assert d.lp_p010 == _abi.LP_P010_TRUNCATE == hdr2sdr.TonemapParams().to_c().lp_p010


@pytest.mark.parametrize('name', sorted(RULES['preview']))
def test_preview_chains_parse(name):
    """The reference's preview -vf strings (FFMPEG_FILTER with PREVIEW_SIZE;
    build_libplacebo_filter with numeric w/h, src/utils.py:787) parse to the
    params Previewer chooses for the same request, with the box."""
    chain = RULES['preview'][name]
    params, lut, box = PV.parse_preview_chain(chain)
    assert box == (3840, 2160)
    kind, tm = name.split('_')[:2]
    lut_on = not name.endswith('lut0')
    want = PV.preview_params(tm, lut_enabled=lut_on, use_gpu=kind == 'gpu')
    keys = ('tonemapper', 'gamma', 'bits_out', 'lut_enabled', 'peak_detect', 'desat', 'lp_p010')
    assert {k: getattr(params, k) for k in keys} == {k: getattr(want, k) for k in keys}
    assert params.resolved_pipeline() == want.resolved_pipeline()
    assert (lut == '<LUT>') == lut_on


def test_preview_selects_the_reference_chain():
    """src/preview.py:584-590: libplacebo for GPU-only operators always and
    for every operator when GPU tone mapping is on; the CPU preview honours
    lut_enabled through the legacy chain."""
    assert PV.preview_params('bt.2390').resolved_pipeline() == 'libplacebo'
    assert PV.preview_params('bt.2390').peak_detect
    assert PV.preview_params('hable').resolved_pipeline() == 'cpu'
    assert PV.preview_params('hable', use_gpu=True).resolved_pipeline() == 'libplacebo'
    assert not PV.preview_params('hable', lut_enabled=False).lut_enabled
    with pytest.raises(ValueError):
        PV.parse_preview_chain('zscale=t=linear:npl=100,tonemap=hable,zscale=t=bt709:m=bt709:r=tv,'
                               'eq=gamma=1.0,scale=960:540:force_original_aspect_ratio=increase')


def _stub_ns():
    """INTEGRATION.md's reference-side stub, executed (as tests/test_abi_exports.py does)."""
    import re
    from hdr2sdr import _abi
    doc = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'INTEGRATION.md')).read()
    code = re.search(r'```python\n(# src/h2s_backend.py.*?)```', doc, re.S).group(1)
    old = os.environ.get('H2S_LIB')
    os.environ['H2S_LIB'] = _abi.LIB_PATH
    try:
        ns = {}
        exec(compile(code, 'INTEGRATION.md', 'exec'), ns)
    finally:
        if old is None:
            del os.environ['H2S_LIB']
        else:
            os.environ['H2S_LIB'] = old
    return ns


@pytest.mark.parametrize('case', [c for c in RULES['cases'] if c.get('libplacebo', True)], ids=_case_id)
def test_integration_stub_follows_the_same_rules(case):
    """The stub a maintainer adds (src/h2s_backend.py) builds the same
    h2s_params as from_request for every captured case, and raises the same
    ValueError (the stub takes libplacebo as available: libh2s runs it)."""
    ns = _stub_ns()
    interop = case.get('encoder') == 'h264_nvenc' and case.get('interop', False)
    props = case.get('props', {})
    if _dovi5(case) and 'error' not in case:
        with pytest.raises(ValueError) as e:
            ns['params_for'](Req(**case['req']), 10, props, interop)
        assert str(e.value) == C.DOVI_P5_ERROR
        return
    if 'error' in case:
        with pytest.raises(ValueError) as e:
            ns['params_for'](Req(**case['req']), 10, props, interop)
        assert str(e.value) == case['error']
        return
    got = ns['params_for'](Req(**case['req']), 10, props, interop)
    p, _ = _from_request(case)
    want = p.to_c()
    import ctypes
    assert bytes(memoryview(got)) == bytes(memoryview(want)) or all(
        (getattr(got, n) == getattr(want, n)) or (getattr(got, n) != getattr(got, n) and getattr(want, n) != getattr(want, n))
        for n, _ in want._fields_ if n != 'reserved'), {n: (getattr(got, n), getattr(want, n)) for n, _ in want._fields_}
    assert ctypes.sizeof(got) == ctypes.sizeof(want)
