"""The reference-facing interface: chain strings, requests, tone-map names.
Pinned against filter_chains.json, captured from the reference's own
ffmpeg_command.build() / _filter_args (tests/golden/make_golden.py).
Mirrors test/ffmpeg_command_test.py TestFilterArgs (:195-235)."""
import json
import math
import os
from dataclasses import dataclass

import pytest

import hdr2sdr
from hdr2sdr.chain import parse_filter_chain


@pytest.fixture(scope='module')
def chains(golden_dir):
    with open(os.path.join(golden_dir, 'filter_chains.json')) as f:
        return json.load(f)


@dataclass(frozen=True)
class Req:  # a RequestLike (src/ffmpeg_command.py:54-85)
    input_path: str = 'in.mkv'
    output_path: str = 'out.mkv'
    gamma: float = 1.0
    use_gpu: bool = False
    tonemapper: str = 'reinhard'
    quality: int = 23
    quality_mode: str = 'cq'
    bit_depth: int = 8
    licensed: bool = False
    lut_enabled: bool = True


def test_constants_match_reference(chains):
    assert hdr2sdr.FFMPEG_CONVERT_FILTER == chains['FFMPEG_CONVERT_FILTER']
    assert hdr2sdr.TONEMAP == chains['TONEMAP']
    assert sorted(hdr2sdr.GPU_ONLY_TONEMAPPERS) == chains['GPU_ONLY_TONEMAPPERS']
    assert hdr2sdr.is_gpu_only_tonemapper('BT.2390') and not hdr2sdr.is_gpu_only_tonemapper('Hable')


@pytest.mark.parametrize('case,tm,gamma,bits_out', [
    ('C1', 'reinhard', 1.0, 10), ('C2', 'hable', 2.2, 10), ('C4', 'mobius', 1.0, 10),
    ('C5', 'hable', 1.0, 12), ('default8', 'mobius', 1.0, 8), ('gamma05', 'hable', 0.5, 8)])
def test_reference_cpu_chains_parse(chains, case, tm, gamma, bits_out):
    c = chains[case]
    p, lut = parse_filter_chain(c['filter_complex'], bits_out=bits_out)
    assert (p.tonemapper, p.gamma, p.lut_enabled, p.npl, p.desat) == (tm, gamma, True, 100.0, 2.0)
    assert math.isnan(p.tm_param) and p.peak == 0.0
    assert lut == '<LUT>'
    # and the request path lands on the same params + the same string
    r = Req(**{**c['request'], 'tonemapper': c['request']['tonemapper'].lower()})
    q = hdr2sdr.TonemapParams.from_request(r)
    assert (q.tonemapper, q.gamma, q.bits_out) == (tm, gamma, bits_out)
    pix = {8: 'yuv420p', 10: 'yuv420p10le', 12: 'yuv420p12le'}[q.bits_out]
    assert pix == c['pix_fmt']
    assert '[0:v:0]' + q.filter_string() + '[vout]' == c['filter_complex']


def test_libplacebo_chain_parses_to_native_bt2390(chains):
    p, lut = parse_filter_chain(chains['C3']['filter_complex'])
    assert p.tonemapper == 'bt.2390' and p.lut_enabled and p.desat == 0.0 and lut == '<LUT>'


def test_cpu_chain_refuses_gpu_only_operator(chains):
    with pytest.raises(ValueError) as e:
        hdr2sdr.TonemapParams(tonemapper='bt.2390').filter_string()
    assert 'requires GPU tonemapping' in str(e.value)
    assert 'requires GPU tonemapping' in chains['cpu_bt2390_error']


def test_legacy_no_lut_chain(chains):
    legacy = chains['FFMPEG_FILTER_LEGACY_NO_LUT'].replace(
        ',scale={width}:{height}:force_original_aspect_ratio=decrease', '')
    p, lut = parse_filter_chain(legacy.format(gamma=1.5, tonemapper='hable'))
    assert not p.lut_enabled and lut is None and p.gamma == 1.5


def test_tonemap_options_and_errors():
    p, _ = parse_filter_chain('zscale=t=linear:npl=200,tonemap=tonemap=reinhard:param=0.25:desat=0:peak=12,'
                              'zscale=t=bt709,eq=gamma=1.1')
    assert (p.tonemapper, p.tm_param, p.desat, p.peak, p.npl, p.lut_enabled) == \
        ('reinhard', 0.25, 0.0, 12.0, 200.0, False)
    for bad in ('tonemap=hable', 'zscale=t=linear,tonemap=hable,scale=640:360',
                'zscale=t=linear,tonemap=hable,lut3d=file=x.cube:interp=trilinear',
                'zscale=t=linear,tonemap=spline', 'zscale=t=linear,tonemap=hable,eq=contrast=2'):
        with pytest.raises(ValueError):
            parse_filter_chain(bad)


def test_params_validation_and_struct():
    # spline is a native operator now (libplacebo's curve, restated); its
    # contrast param is range-checked as pl_tone_map_spline declares (0..1.5)
    assert hdr2sdr.TonemapParams(tonemapper='Spline').to_c().tonemap == 8
    with pytest.raises(ValueError):
        hdr2sdr.TonemapParams(tonemapper='spline', tm_param=2.0)
    with pytest.raises(ValueError):
        hdr2sdr.TonemapParams(tonemapper='spline').filter_string()   # GPU-only, as in the reference
    with pytest.raises(ValueError):
        hdr2sdr.TonemapParams(tonemapper='unknown')
    with pytest.raises(ValueError):
        hdr2sdr.TonemapParams(bits_in=8)
    with pytest.raises(ValueError):
        hdr2sdr.TonemapParams(gamma=0)
    c = hdr2sdr.TonemapParams(tonemapper='Hable', gamma=2.2, bits_out=12, transfer='arib-std-b67',
                              mode='native').to_c()
    assert (c.tonemap, c.transfer_in, c.bits_out, c.mode, c.lut_enabled) == (5, 1, 12, 1, 1)
    # from_request: 12-bit request -> yuv420p12le, CPU chain always applies the LUT
    q = hdr2sdr.TonemapParams.from_request(Req(tonemapper='Mobius', bit_depth=12, lut_enabled=False))
    assert q.bits_out == 12 and q.lut_enabled and q.tonemapper == 'mobius'


def test_libplacebo_spline_chain_parses_to_native_spline():
    """build_libplacebo_filter (src/utils.py:392-471) with tonemapping=spline,
    as the reference builds it for a GPU-only operator."""
    chain = ('[0:v:0]format=p010,hwupload,libplacebo=w=iw:h=ih:tonemapping=spline:colorspace=bt709:'
             'color_primaries=auto:color_trc=bt709:range=tv:peak_detect=1:format=rgba,hwdownload,format=rgba,'
             'lut3d=file=<LUT>:interp=tetrahedral,setparams=color_primaries=bt709:color_trc=bt709:'
             'colorspace=bt709[vout]')
    p, lut = parse_filter_chain(chain)
    assert p.tonemapper == 'spline' and p.peak_detect and p.desat == 0.0 and p.lut_enabled and lut == '<LUT>'


@pytest.mark.parametrize('tm', ['hable', 'mobius', 'reinhard'])
def test_libplacebo_chain_with_cpu_operator_names_parses(tm):
    """The reference emits a libplacebo chain for every operator when GPU
    tone mapping is on (src/ffmpeg_command.py:119, :236): libplacebo's own
    reinhard / hable / mobius (NORM scaling, restated) on the libplacebo
    pipeline, not vf_tonemap's curves of the same name."""
    chain = (f'[0:v:0]format=p010,hwupload,libplacebo=w=iw:h=ih:tonemapping={tm}:colorspace=bt709:'
             'color_primaries=auto:color_trc=bt709:range=tv:peak_detect=1:format=rgba,hwdownload,format=rgba,'
             'lut3d=file=<LUT>:interp=tetrahedral,setparams=color_primaries=bt709:color_trc=bt709:'
             'colorspace=bt709[vout]')
    p, _ = parse_filter_chain(chain)
    assert p.tonemapper == tm and p.pipeline == 'libplacebo' and p.peak_detect and p.desat == 0.0


@pytest.mark.parametrize('tm', ['clip', 'linear', 'gamma'])
def test_libplacebo_chain_with_other_operators_is_rejected(tm):
    chain = f'libplacebo=w=iw:h=ih:tonemapping={tm}:peak_detect=1:format=rgba,hwdownload,format=rgba'
    with pytest.raises(ValueError):
        parse_filter_chain(chain)


# ---- the libplacebo stage: only the option values the engine models ---------
_LP = ('format=p010,hwupload,libplacebo=w=iw:h=ih:tonemapping=bt.2390:colorspace=bt709:'
       'color_primaries={prim}:color_trc=bt709:range={rng}:peak_detect=1:format={fmt}{extra},'
       'hwdownload,format={fmt}{lut}')
_LUT = ',lut3d=file=<LUT>:interp=tetrahedral,setparams=color_primaries=bt709:color_trc=bt709:colorspace=bt709'


def _lp(prim='auto', rng='tv', fmt='rgba', extra='', lut=_LUT):
    return _LP.format(prim=prim, rng=rng, fmt=fmt, extra=extra, lut=lut)


def test_libplacebo_reference_options_parse():
    """Both forms build_libplacebo_filter emits (src/utils.py:445-449): LUT
    on (primaries auto, rgba) and off (bt709, nv12)."""
    p, lut = hdr2sdr.parse_filter_chain(_lp())
    assert p.pipeline == 'libplacebo' and p.lut_enabled and lut == '<LUT>' and p.peak_detect
    assert p.lp_range == 'full'
    p, lut = hdr2sdr.parse_filter_chain(_lp(prim='bt709', fmt='nv12', lut=''))
    assert not p.lut_enabled and lut is None
    p, _ = hdr2sdr.parse_filter_chain(_lp(rng='pc'))      # full range: no model choice left
    assert p.lp_range == 'full'
    p, _ = hdr2sdr.parse_filter_chain(_lp(), lp_range='limited')   # range=tv follows the model switch
    assert p.lp_range == 'limited'


@pytest.mark.parametrize('chain', [
    _lp(rng='jpeg'),                                   # range value not modelled
    _lp(extra=':dithering=blue'),                      # option not modelled
    _lp(extra=':percentile=99.9'),                     # peak-detect options are h2s_params fields, not parsed
    _lp().replace('color_trc=bt709', 'color_trc=smpte2084'),
    _lp().replace('colorspace=bt709', 'colorspace=bt2020nc'),
    _lp().replace('w=iw', 'w=wide'),                   # a size expression libplacebo would evaluate
    _lp(prim='bt709'),                                 # libplacebo gamut mapping and the LUT: a double conversion
    _lp(prim='auto', fmt='nv12', lut=''),              # no gamut conversion at all
])
def test_libplacebo_unmodelled_options_are_rejected(chain):
    with pytest.raises(ValueError):
        hdr2sdr.parse_filter_chain(chain)


def test_libplacebo_numeric_size_is_the_previews_box():
    """extract_frame_with_gpu_conversion passes PREVIEW_SIZE as w/h
    (src/utils.py:787): that is the Previewer's box (parse_preview_chain),
    while a conversion chain with a numeric size is rejected, since the
    engine runs conversions at the source size and would silently ignore it
    (build() only ever emits w=iw:h=ih, src/utils.py:446)."""
    from hdr2sdr import preview as PV
    chain = _lp().replace('w=iw:h=ih', 'w=1920:h=1080')
    with pytest.raises(ValueError):
        parse_filter_chain(chain)
    p, lut, box = PV.parse_preview_chain(chain)
    assert p.resolved_pipeline() == 'libplacebo' and p.peak_detect and lut == '<LUT>'
    assert box == (1920, 1080)