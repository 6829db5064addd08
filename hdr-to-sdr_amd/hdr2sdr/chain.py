"""The reference's filter-chain interface, mirrored.

The reference selects its hot path as a string: ``FFMPEG_CONVERT_FILTER``
(src/utils.py:38-42) formatted with ``gamma``, ``tonemapper`` and the LUT path
by ``ffmpeg_command._filter_args`` (src/ffmpeg_command.py:227-247), from the
fields of ``ConversionRequest`` (src/conversion.py:26-44).  This module keeps
those names and semantics and turns either a request or a chain string into
the ``TonemapParams`` the HIP engine executes:

* ``TONEMAP`` / ``GPU_ONLY_TONEMAPPERS`` / ``is_gpu_only_tonemapper`` —
  src/utils.py:16, :67-73.
* ``FFMPEG_CONVERT_FILTER`` — src/utils.py:38-42 (the same template, so a
  chain built by the reference parses here unchanged).
* ``TonemapParams.from_request`` — what ``_filter_args`` + ``_codec_and_pix_fmt``
  decide for one request (tonemapper lower-cased :235, pix_fmt :355-360).
* ``parse_filter_chain`` — the drop-in: any chain string the reference
  builds (CPU chain, legacy no-LUT preview chain) maps onto one kernel launch.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, replace
from typing import Any, Callable

from . import _abi

# src/utils.py:16
TONEMAP = ["Reinhard", "Mobius", "Hable", "BT.2390", "Spline"]

# src/utils.py:38-42 (template kept verbatim: it is the interface)
FFMPEG_CONVERT_FILTER = (
    'zscale=t=linear:npl=100,tonemap={tonemapper},zscale=t=bt709:m=bt709:r=tv,'
    'lut3d=file={lut_path}:interp=tetrahedral,setparams=color_primaries=bt709:color_trc=bt709:colorspace=bt709,'
    'eq=gamma={gamma}'
)

# src/utils.py:67.  The reference can only run these through libplacebo; this
# engine runs both natively on the GPU (BT.2390 EETF and libplacebo's spline
# curve, restated in libh2s; parity unpinned).
GPU_ONLY_TONEMAPPERS = {'bt.2390', 'spline'}
# every operator of the reference's TONEMAP list reaches libplacebo when GPU
# tone mapping is on (src/utils.py:16; src/ffmpeg_command.py:236-239)
LIBPLACEBO_TONEMAPPERS = {'reinhard', 'mobius', 'hable', 'bt.2390', 'spline'}

_TM_NAMES = {
    'none': _abi.TM_NONE, 'linear': _abi.TM_LINEAR, 'gamma': _abi.TM_GAMMA,
    'clip': _abi.TM_CLIP, 'reinhard': _abi.TM_REINHARD, 'hable': _abi.TM_HABLE,
    'mobius': _abi.TM_MOBIUS, 'bt.2390': _abi.TM_BT2390, 'bt2390': _abi.TM_BT2390,
    'spline': _abi.TM_SPLINE,
}
_TRC_NAMES = {'smpte2084': _abi.TRC_PQ, 'pq': _abi.TRC_PQ,
              'arib-std-b67': _abi.TRC_HLG, 'hlg': _abi.TRC_HLG}
_MODES = {'compat8': _abi.MODE_COMPAT8, 'native': _abi.MODE_NATIVE}
_DESAT_LUMA = {'rgb': _abi.DESAT_LUMA_RGB, 'bt2020': _abi.DESAT_LUMA_BT2020,
               'bt709': _abi.DESAT_LUMA_BT709}
# [EXT] switches (include/h2s.h)
_CHROMA = {'box': _abi.CHROMA_BOX, 'bicubic': _abi.CHROMA_BICUBIC}
_DITHER = {'none': _abi.DITHER_NONE, 'ordered': _abi.DITHER_ORDERED}
_EXPAND = {'shift': _abi.EXPAND_SHIFT, 'replicate': _abi.EXPAND_REPLICATE}
# which of the reference's two chains: 'auto' = libplacebo for the GPU-only
# operators (the only chain that has them), the CPU chain otherwise
_LUT_IN = {'float': _abi.LUT_IN_FLOAT, 'rgb48': _abi.LUT_IN_RGB48}
_LP_TONE = {'ipt': _abi.LP_TONE_IPT, 'max-rgb': _abi.LP_TONE_MAX_RGB}
_EDGE = {'zimg': _abi.EDGE_ZIMG, 'replicate': _abi.EDGE_REPLICATE, 'mirror': _abi.EDGE_MIRROR}
_PIPELINE = {'auto': _abi.PIPE_AUTO, 'cpu': _abi.PIPE_CPU_CHAIN, 'libplacebo': _abi.PIPE_LIBPLACEBO}
# libplacebo stage options (include/h2s.h enum h2s_lp_range / _dither / _p010)
_LP_RANGE = {'full': _abi.LP_RANGE_FULL, 'limited': _abi.LP_RANGE_LIMITED}
_LP_DITHER = {'none': _abi.LP_DITHER_NONE, 'ordered': _abi.LP_DITHER_ORDERED}
_LP_P010 = {'keep': _abi.LP_P010_KEEP, 'truncate': _abi.LP_P010_TRUNCATE}


def is_gpu_only_tonemapper(tonemapper: str) -> bool:
    """src/utils.py:70-73: case-insensitive membership test."""
    return tonemapper.lower() in GPU_ONLY_TONEMAPPERS


# src/ffmpeg_command.py:241-245 (the message _filter_args raises)
CPU_GPU_ONLY_ERROR = ("{tonemapper} requires GPU tonemapping; this item's settings force CPU processing "
                      "— change the tonemapper or output bit depth.")


# Dolby Vision profile 5 (src/ffmpeg_command.py:100-106, :117-128): the
# reference routes it to libplacebo because libplacebo applies the RPU
# (reshaping + the IPT-PQ-c2 colour matrix carried as side data); without it
# "the output colors may look wrong (green/purple cast)".  The rawvideo pipe
# the drop-in reads drops every side-data packet, so no RPU can reach libh2s:
# the drop-in refuses such a source and the caller keeps the reference's own
# command
DOVI_P5_ERROR = ("Dolby Vision profile 5 needs its RPU (applied by libplacebo in the reference, "
                 "src/ffmpeg_command.py:100-106); the rawvideo pipe drops it, so libh2s cannot convert "
                 "this source — keep the reference command.")


def is_dovi_profile5(properties: 'dict[str, Any] | None') -> bool:
    """``_tonemap_plan``'s test (src/ffmpeg_command.py:104-106)."""
    props = properties or {}
    return bool(props.get('is_dolby_vision') and props.get('dovi_profile') == 5)


@dataclass(frozen=True)
class TonemapPlan:
    """The branch decision of ``_tonemap_plan`` (src/ffmpeg_command.py:87-93,
    :96-144), without its notices (UI, out of scope)."""
    use_gpu: bool
    dovi_needs_rpu: bool
    use_libplacebo: bool


def tonemap_plan(request: Any, properties: 'dict[str, Any] | None' = None,
                 libplacebo_available: 'bool | Callable[[], bool]' = True) -> TonemapPlan:
    """src/ffmpeg_command.py:96-144: bit_depth >= 12 turns ``use_gpu`` off
    (no 12-bit hardware HEVC profile); Dolby Vision profile 5 needs the RPU
    libplacebo applies, so it forces libplacebo even without ``use_gpu``;
    the libplacebo probe is consulted only when one of the two asks for it
    (the reference's laziness: a callable is called at most once, and only
    then)."""
    use_gpu = bool(getattr(request, 'use_gpu', False))
    if int(getattr(request, 'bit_depth', 8)) >= 12:
        use_gpu = False
    dovi = is_dovi_profile5(properties)
    use_lp = False
    if use_gpu or dovi:
        use_lp = bool(libplacebo_available() if callable(libplacebo_available) else libplacebo_available)
    return TonemapPlan(use_gpu=use_gpu, dovi_needs_rpu=dovi, use_libplacebo=use_lp)


@dataclass(frozen=True)
class TonemapParams:
    """Everything one kernel launch needs besides the LUT lattice.

    Defaults are the reference chain's: npl=100, vf_tonemap's desat 2.0 and
    automatic peak, tetrahedral LUT on, eq gamma 1.0, and the settings
    defaults (src/settings.py:10-26: Mobius)."""
    tonemapper: str = 'mobius'
    gamma: float = 1.0
    bits_in: int = 10
    bits_out: int = 10
    transfer: str = 'smpte2084'
    lut_enabled: bool = True
    mode: str = 'compat8'
    tm_param: float = math.nan
    desat: float = 2.0
    peak: float = 0.0
    npl: float = 100.0
    maxcll: float = 0.0
    mastering_max: float = 0.0
    desat_luma: str = 'rgb'
    peak_detect: bool = False   # BT.2390 / spline: detected, smoothed per-frame peak (libplacebo peak_detect=1)
    chroma_filter: str = 'box'  # S6 4:4:4 -> 4:2:0 ('box' | 'bicubic')
    dither: str = 'none'        # 8-bit quantiser ('none' | 'ordered')
    expand: str = 'shift'       # S8 8-bit -> bits_out ('shift' | 'replicate')
    pipeline: str = 'auto'      # 'cpu' (FFMPEG_CONVERT_FILTER) | 'libplacebo' (build_libplacebo_filter) | 'auto'
    knee_offset: float = math.nan   # BT.2390 knee offset (NaN: libplacebo's 1.0; 0.5 = ITU-R BT.2390)
    target_black: float = math.nan  # SDR target black, nits (NaN: pipeline default)
    target_white: float = math.nan  # SDR target white, nits (NaN: libplacebo 203, CPU chain npl)
    chroma_edge: str = 'zimg'   # S1 upsampler edge rule ('zimg' | 'replicate' | 'mirror')
    lut_input: str = 'float'    # S3 -> S4 format on the CPU chain ('float' | 'rgb48')
    lp_tone: str = 'ipt'        # libplacebo branch: curve on IPT intensity | gain on max(R,G,B) ('ipt' | 'max-rgb')
    # libplacebo branch options (include/h2s.h ABI v3; PARITY UNPINNED models)
    lp_range: str = 'full'      # what range=tv does to the rgba download ('full' | 'limited')
    lp_dither: str = 'none'     # the 8-bit download ('none' | 'ordered')
    # 12-bit input through the upload prefix: 'truncate' = format=p010,hwupload
    # (the reference's default, src/utils.py:431), 'keep' = the CUDA-interop
    # hwmap=derive_device=vulkan prefix (:430)
    lp_p010: str = 'truncate'
    # peak_detect=1 parameters (NaN: vf_libplacebo's defaults 100 / 5.5 / 10 / 99.995 / 1.0)
    pd_smoothing: float = math.nan
    pd_scene_low: float = math.nan
    pd_scene_high: float = math.nan
    pd_percentile: float = math.nan
    pd_min_peak: float = math.nan

    def __post_init__(self) -> None:
        tm = self.tonemapper.lower()
        if tm not in _TM_NAMES:
            raise ValueError(f'unknown tonemapper {self.tonemapper!r}')
        if self.transfer not in _TRC_NAMES:
            raise ValueError(f'unknown input transfer {self.transfer!r}')
        if self.mode not in _MODES:
            raise ValueError(f'unknown mode {self.mode!r}')
        if self.desat_luma not in _DESAT_LUMA:
            raise ValueError(f'unknown desat_luma {self.desat_luma!r}')
        for name, table in (('chroma_filter', _CHROMA), ('dither', _DITHER), ('expand', _EXPAND),
                            ('pipeline', _PIPELINE), ('chroma_edge', _EDGE), ('lut_input', _LUT_IN), ('lp_tone', _LP_TONE),
                            ('lp_range', _LP_RANGE), ('lp_dither', _LP_DITHER), ('lp_p010', _LP_P010)):
            if getattr(self, name) not in table:
                raise ValueError(f'unknown {name} {getattr(self, name)!r}; expected one of {sorted(table)}')
        if self.pipeline == 'libplacebo' and tm not in LIBPLACEBO_TONEMAPPERS:
            raise ValueError(f'libplacebo tonemapping={tm} is not supported '
                             f'(the reference names {sorted(LIBPLACEBO_TONEMAPPERS)})')
        if self.bits_in not in (10, 12):
            raise ValueError(f'bits_in must be 10 or 12, got {self.bits_in}')
        if self.bits_out not in (8, 10, 12):
            raise ValueError(f'bits_out must be 8, 10 or 12, got {self.bits_out}')
        if not self.gamma > 0:
            raise ValueError(f'gamma must be > 0, got {self.gamma}')
        if tm == 'spline' and not math.isnan(self.tm_param) and not 0.0 <= self.tm_param <= 1.5:
            # libplacebo pl_tone_map_spline: param_min 0, param_max 1.5 (contrast)
            raise ValueError(f'spline contrast (tm_param) must be in [0, 1.5], got {self.tm_param}')

    # ---- construction from the reference's request ---------------------
    @classmethod
    def from_request(cls, request: Any, bits_in: int = 10, transfer: str = 'smpte2084',
                     properties: 'dict[str, Any] | None' = None,
                     libplacebo_available: 'bool | Callable[[], bool]' = True,
                     cuda_interop: bool = False, **overrides: Any) -> 'TonemapParams':
        """Map a ConversionRequest-like object (src/conversion.py:26-44) to
        the params of the chain the reference's build() would emit for it.

        * the branch: ``tonemap_plan`` (src/ffmpeg_command.py:96-144):
          ``use_gpu`` sends every operator through libplacebo, bit_depth >= 12
          forces the CPU chain; Dolby Vision profile 5 (which the reference
          sends to libplacebo for its RPU) raises ``ValueError`` with
          ``DOVI_P5_ERROR``: the RPU cannot cross the rawvideo pipe, so the
          caller keeps the reference command;
        * CPU chain (src/ffmpeg_command.py:240-247): bt.2390 / spline raise
          ``ValueError`` with the reference's message; the LUT is always on
          (``lut_enabled`` is ignored there, as ``_filter_args`` ignores it);
        * libplacebo branch (``build_libplacebo_filter``, src/utils.py:392-471):
          ``peak_detect=1`` always (:398, :448), ``lut_enabled`` honoured
          (:435, :444, :451), and the upload prefix ``format=p010,hwupload``
          (12-bit input cut to p010's 10 bits, ``lp_p010`` truncate) unless the
          CUDA-interop ``hwmap`` prefix is used (``cuda_interop``: keep), :430-431;
        * tonemapper lower-cased (src/ffmpeg_command.py:235); bit_depth ->
          output depth (src/ffmpeg_command.py:355-360; 8 -> yuv420p).
        ``properties`` / ``libplacebo_available`` are build()'s probe inputs
        (``Probes.resolve_libplacebo_available``, src/ffmpeg_command.py:431-452):
        the engine itself always runs the libplacebo branch natively, so the
        default is True."""
        plan = tonemap_plan(request, properties, libplacebo_available)
        if plan.dovi_needs_rpu:
            raise ValueError(DOVI_P5_ERROR)
        tm = str(request.tonemapper).lower()
        bit_depth = int(getattr(request, 'bit_depth', 8))
        bits_out = 12 if bit_depth >= 12 else (10 if bit_depth == 10 else 8)
        kw: 'dict[str, Any]' = dict(tonemapper=tm, gamma=float(request.gamma), bits_in=bits_in,
                                    bits_out=bits_out, transfer=transfer)
        if plan.use_libplacebo:
            if tm not in LIBPLACEBO_TONEMAPPERS:
                raise ValueError(f'libplacebo tonemapping={tm} is not supported '
                                 f'(the reference names {sorted(LIBPLACEBO_TONEMAPPERS)})')
            kw.update(pipeline='libplacebo', desat=0.0, peak_detect=True,
                      lut_enabled=bool(getattr(request, 'lut_enabled', True)),
                      lp_p010='keep' if cuda_interop else 'truncate')
        else:
            if is_gpu_only_tonemapper(tm):
                raise ValueError(CPU_GPU_ONLY_ERROR.format(tonemapper=tm))
            kw.update(pipeline='cpu', lut_enabled=True)
        kw.update(overrides)
        return cls(**kw)

    def with_(self, **kw: Any) -> 'TonemapParams':
        return replace(self, **kw)

    # ---- C struct ---------------------------------------------------------
    def to_c(self) -> _abi.H2SParams:
        p = _abi.H2SParams()
        p.transfer_in = _TRC_NAMES[self.transfer]
        p.bits_in = self.bits_in
        p.bits_out = self.bits_out
        p.tonemap = _TM_NAMES[self.tonemapper.lower()]
        p.tm_param = self.tm_param
        p.desat = self.desat
        p.peak = self.peak
        p.npl = self.npl
        p.gamma = self.gamma
        p.maxcll = self.maxcll
        p.mastering_max = self.mastering_max
        p.lut_enabled = 1 if self.lut_enabled else 0
        p.mode = _MODES[self.mode]
        p.desat_luma = _DESAT_LUMA[self.desat_luma]
        p.peak_detect = 1 if self.peak_detect else 0
        p.chroma_filter = _CHROMA[self.chroma_filter]
        p.dither = _DITHER[self.dither]
        p.expand = _EXPAND[self.expand]
        p.pipeline = _PIPELINE[self.pipeline]
        p.knee_offset = self.knee_offset
        p.target_black = self.target_black
        p.target_white = self.target_white
        p.chroma_edge = _EDGE[self.chroma_edge]
        p.lut_input = _LUT_IN[self.lut_input]
        p.lp_tone = _LP_TONE[self.lp_tone]
        p.lp_range = _LP_RANGE[self.lp_range]
        p.lp_dither = _LP_DITHER[self.lp_dither]
        p.lp_p010 = _LP_P010[self.lp_p010]
        p.pd_smoothing = self.pd_smoothing
        p.pd_scene_low = self.pd_scene_low
        p.pd_scene_high = self.pd_scene_high
        p.pd_percentile = self.pd_percentile
        p.pd_min_peak = self.pd_min_peak
        return p

    def resolved_pipeline(self) -> str:
        """'cpu' or 'libplacebo' after 'auto' resolution."""
        if self.pipeline != 'auto':
            return self.pipeline
        return 'libplacebo' if is_gpu_only_tonemapper(self.tonemapper) else 'cpu'

    # ---- back to the reference's chain string --------------------------
    def filter_string(self, lut_path: str = '<LUT>', width: 'int | str' = 'iw', height: 'int | str' = 'ih') -> str:
        """The chain the reference would build for these params: the CPU
        chain (FFMPEG_CONVERT_FILTER.format, src/ffmpeg_command.py:246-247),
        or for ``pipeline='libplacebo'`` the string of ``build_libplacebo_filter``
        (src/utils.py:392-471) with the upload prefix ``lp_p010`` stands for
        (truncate: ``format=p010,hwupload``; keep: the CUDA-interop ``hwmap``)."""
        if self.pipeline == 'libplacebo':
            return self._libplacebo_string(lut_path, width, height)
        if is_gpu_only_tonemapper(self.tonemapper):
            # src/ffmpeg_command.py:240-245
            raise ValueError(f"{self.tonemapper.lower()} requires GPU tonemapping; the reference CPU chain "
                             "has no equivalent")
        return FFMPEG_CONVERT_FILTER.format(gamma=self.gamma, tonemapper=self.tonemapper.lower(),
                                            lut_path=lut_path)

    def _libplacebo_string(self, lut_path: str, width: 'int | str', height: 'int | str') -> str:
        # the stage order and options of src/utils.py:426-471, composed from
        # this engine's own fields (only the chain string is the interface)
        interop = self.lp_p010 == 'keep'
        lut = self.lut_enabled
        fmt = 'rgba' if lut else 'nv12'
        stage = (f'libplacebo=w={width}:h={height}:tonemapping={self.tonemapper.lower()}:colorspace=bt709:'
                 f'color_primaries={"auto" if lut else "bt709"}:color_trc=bt709:range=tv:'
                 f'peak_detect={1 if self.peak_detect else 0}:format={fmt}')
        parts = ['hwmap=derive_device=vulkan' if interop else 'format=p010,hwupload', stage]
        identity = abs(self.gamma - 1.0) < 1e-9
        if lut:
            parts += ['hwdownload', f'format={fmt}', f'lut3d=file={lut_path}:interp=tetrahedral',
                      'setparams=color_primaries=bt709:color_trc=bt709:colorspace=bt709']
        elif interop and identity:
            parts += ['hwmap=reverse=1:derive_device=cuda']
        else:
            parts += ['hwdownload', 'format=nv12']
        if not identity:
            parts.append(f'eq=gamma={self.gamma}')
        return ','.join(parts)


_WRAP = re.compile(r'^\s*\[[^\]]*\](.*?)\[[^\]]*\]\s*$')


def _split_filters(chain: str) -> 'list[tuple[str, dict[str, str], list[str]]]':
    """Split 'name=a=1:b=2,name2=v' into (name, {key: value}, [positional])."""
    out = []
    for part in re.split(r',(?![^\[]*\])', chain):
        part = part.strip()
        if not part:
            continue
        name, _, args = part.partition('=')
        kv: 'dict[str, str]' = {}
        pos: 'list[str]' = []
        # split on ':' not preceded by a backslash (escaped drive colons)
        for tok in re.split(r'(?<!\\):', args) if args else []:
            if '=' in tok:
                k, _, v = tok.partition('=')
                kv[k.strip()] = v.strip()
            else:
                pos.append(tok.strip())
        out.append((name.strip(), kv, pos))
    return out


# libplacebo stage options build_libplacebo_filter emits (src/utils.py:445-449)
# and the values the engine models; anything else is rejected rather than
# converted with a behaviour the string did not ask for
_LP_OPTION_VALUES = {
    # output size: build() emits w=iw:h=ih for a conversion (src/utils.py:446):
    # the engine runs the chain at the source size, so a numeric size would be
    # silently ignored and is rejected.  The preview's numbers
    # (extract_frame_with_gpu_conversion passes PREVIEW_SIZE, src/utils.py:787)
    # are the Previewer's box: parse_preview_chain takes them out first
    'w': {'iw'}, 'h': {'ih'},
    'colorspace': {'bt709'},
    'color_primaries': {'auto', 'bt709'},      # with / without the lut3d stage (checked after the loop)
    'color_trc': {'bt709'},
    'range': {'tv', 'pc'},                     # tv: the lp_range model; pc: full range
    'peak_detect': {'0', '1', 'true', 'false'},
    'format': {'rgba', 'nv12'},                # with / without the lut3d stage
}


def _check_libplacebo_options(kv: 'dict[str, str]', pos: 'list[str]') -> None:
    if pos:
        raise ValueError(f'libplacebo positional options {pos} are not modelled')
    for k, v in kv.items():
        if k == 'tonemapping':
            continue
        if k not in _LP_OPTION_VALUES:
            raise ValueError(f'libplacebo option {k}={v} is not modelled '
                             f'(the reference sets {sorted(_LP_OPTION_VALUES)} and tonemapping)')
        allowed = _LP_OPTION_VALUES[k]
        if v not in allowed:
            raise ValueError(f'libplacebo {k}={v} is not modelled (accepted: {sorted(allowed)})')


def parse_filter_chain(chain: str, bits_in: int = 10, bits_out: int = 10,
                       transfer: str = 'smpte2084', **overrides: Any) -> 'tuple[TonemapParams, str | None]':
    """Parse a reference chain string into (params, lut_path).

    Accepts FFMPEG_CONVERT_FILTER output (src/utils.py:38-42), the same
    wrapped in build()'s '[0:v:0]...[vout]' (src/ffmpeg_command.py:480-483),
    and the legacy no-LUT chain FFMPEG_FILTER_LEGACY_NO_LUT
    (src/utils.py:57-60; its trailing scale= is a preview resize and is
    rejected here).  Raises ValueError for anything outside the hot path."""
    m = _WRAP.match(chain)
    if m:
        chain = m.group(1)
    kw: 'dict[str, Any]' = dict(bits_in=bits_in, bits_out=bits_out, transfer=transfer,
                                lut_enabled=False)
    lut_path = None
    seen_linear = False
    lp_primaries = lp_format = None
    upload = None   # the libplacebo branch's upload prefix: 'p010' or 'hwmap' (src/utils.py:430-431)
    for name, kv, pos in _split_filters(chain):
        if name == 'zscale':
            t = kv.get('t', kv.get('transfer'))
            if t == 'linear':
                seen_linear = True
                if 'npl' in kv:
                    kw['npl'] = float(kv['npl'])
            elif t == 'bt709':
                if not seen_linear:
                    raise ValueError('zscale=t=bt709 before t=linear')
                # p=bt709 here = the legacy closed-form gamut step
            else:
                raise ValueError(f'unsupported zscale stage {kv}')
        elif name == 'tonemap':
            tm = kv.get('tonemap', pos[0] if pos else None)
            if tm is None:
                raise ValueError('tonemap= without an operator')
            if is_gpu_only_tonemapper(tm):
                # ffmpeg's vf_tonemap has no such operator (src/utils.py:62-66);
                # the reference reaches it only through libplacebo=tonemapping=
                raise ValueError(f'tonemap={tm} does not exist in the CPU chain (libplacebo only)')
            kw['tonemapper'] = tm.lower()
            if 'param' in kv:
                kw['tm_param'] = float(kv['param'])
            if 'desat' in kv:
                kw['desat'] = float(kv['desat'])
            if 'peak' in kv:
                kw['peak'] = float(kv['peak'])
        elif name == 'lut3d':
            interp = kv.get('interp', 'tetrahedral')
            if interp != 'tetrahedral':
                raise ValueError(f'lut3d interp={interp} is not supported (reference uses tetrahedral)')
            lut_path = kv.get('file', pos[0] if pos else None)
            kw['lut_enabled'] = True
        elif name == 'libplacebo':
            # GPU chain build_libplacebo_filter (src/utils.py:392-471): the
            # tone map runs here natively (the libplacebo pipeline: its
            # SDR target, BT.1886 encode, rgba8 download, lut3d 8-bit path).
            tm = kv.get('tonemapping')
            if tm is None:
                raise ValueError('libplacebo stage without tonemapping=')
            if tm.lower() not in LIBPLACEBO_TONEMAPPERS:
                # the reference emits libplacebo chains for each of its five
                # operators with use_gpu (src/ffmpeg_command.py:119, :236;
                # TONEMAP, src/utils.py:16): libplacebo's own reinhard / hable /
                # mobius (NORM scaling) are restated beside bt.2390 / spline
                raise ValueError(f'libplacebo tonemapping={tm} is not supported '
                                 f'(the reference names {sorted(LIBPLACEBO_TONEMAPPERS)})')
            _check_libplacebo_options(kv, pos)
            seen_linear = True
            kw['tonemapper'] = tm.lower()
            kw['desat'] = 0.0
            kw['pipeline'] = 'libplacebo'
            # peak_detect=1 (src/utils.py:448): per-frame detected, temporally
            # smoothed source peak (every libplacebo operator: it sets the source range)
            kw['peak_detect'] = kv.get('peak_detect', '0') in ('1', 'true')
            if kv.get('range') == 'pc':
                kw['lp_range'] = 'full'          # full-range output: no model choice left
            lp_primaries = kv.get('color_primaries')
            lp_format = kv.get('format')
            # format=p010,hwupload: the upload carries 10 bits, so 12-bit input
            # loses its two low bits; the CUDA-interop hwmap prefix keeps them
            if upload is not None:
                kw['lp_p010'] = 'truncate' if upload == 'p010' else 'keep'
        elif name == 'format':
            fmt = kv.get('pix_fmts', pos[0] if pos else None)
            if 'pipeline' not in kw:
                upload = 'p010' if fmt == 'p010' else upload
            continue  # the download's format=rgba / nv12 (src/utils.py:451-460)
        elif name == 'hwmap':
            if 'pipeline' not in kw and kv.get('derive_device') == 'vulkan':
                upload = 'hwmap'
            continue  # Vulkan -> CUDA remap after the stage (src/utils.py:463) moves no pixels
        elif name in ('hwupload', 'hwdownload', 'setparams'):
            continue  # transfers / metadata-only retags (src/utils.py:21-29, :430-460)
        elif name == 'eq':
            if set(kv) - {'gamma'}:
                raise ValueError(f'eq options other than gamma are not supported: {kv}')
            kw['gamma'] = float(kv.get('gamma', 1.0))
        else:
            raise ValueError(f'filter {name!r} is outside the tone-mapping hot path')
    if not seen_linear or 'tonemapper' not in kw:
        raise ValueError('not a tone-mapping chain (needs zscale=t=linear and tonemap=)')
    if kw.get('pipeline') == 'libplacebo':
        # the reference pairs color_primaries=auto + format=rgba with its lut3d
        # stage and color_primaries=bt709 + format=nv12 without it
        # (src/utils.py:432-444); the other pairings are not modelled
        # (absent options take vf_libplacebo's defaults: primaries 'auto' =
        # the input's; format = whatever the following format= filter picks)
        want = ('auto', 'rgba') if kw['lut_enabled'] else ('bt709', 'nv12')
        if (lp_primaries or 'auto') != want[0] or (lp_format or want[1]) != want[1]:
            raise ValueError(f'libplacebo color_primaries={lp_primaries} format={lp_format} with the LUT '
                             f'{"on" if kw["lut_enabled"] else "off"} is not modelled (the reference uses '
                             f'color_primaries={want[0]}:format={want[1]})')
    kw.update(overrides)
    return TonemapParams(**kw), lut_path
