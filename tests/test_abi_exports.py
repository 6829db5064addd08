"""The C-ABI library loads, exports every function include/h2s.h declares,
and the ctypes mirrors of its structs have the C layout.  No compute calls:
runs on the GPU-less build container."""
import ctypes
import os
import re
import subprocess

import pytest

import oracle
from hdr2sdr import _abi

from conftest import REPO, gpu_available

HEADER = os.path.join(REPO, 'include', 'h2s.h')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    names = re.findall(r'^\s*[A-Za-z_][\w\s\*]*?\b(h2s_\w+)\s*\(', src, flags=re.M)
    return sorted(set(names))


def test_header_declares_what_python_binds():
    assert declared_functions() == sorted(_abi.EXPORTS)


def test_library_exports_every_symbol():
    L = ctypes.CDLL(_abi.LIB_PATH)
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(['nm', '-D', '--defined-only', _abi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    for name in declared_functions():
        assert re.search(rf'\bT {name}\b', out), f'{name} not exported as a text symbol'


def test_abi_version_and_defaults():
    L = _abi.lib()
    assert L.h2s_abi_version() == _abi.ABI_VERSION == 3
    assert L.h2s_abi_minor() == _abi.ABI_MINOR == 4
    p = _abi.default_params()
    assert (p.transfer_in, p.bits_in, p.bits_out, p.tonemap, p.desat, p.npl, p.gamma, p.lut_enabled) == \
        (0, 10, 10, 6, 2.0, 100.0, 1.0, 1)
    assert p.tm_param != p.tm_param  # NaN = filter default
    # [EXT] switches default to the round-1 models; libplacebo targets NaN = branch default
    assert (p.chroma_filter, p.dither, p.expand, p.pipeline, p.chroma_edge, p.lut_input) == (0, 0, 0, 0, 0, 0)
    assert p.lp_tone == _abi.LP_TONE_IPT
    for v in (p.knee_offset, p.target_black, p.target_white):
        assert v != v


PROBE = r'''
#include <stddef.h>
#include <stdio.h>
#include "h2s.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(h2s_params), offsetof(h2s_params, tm_param),
         offsetof(h2s_params, lut_enabled), offsetof(h2s_params, desat_luma), sizeof(h2s_frames),
         offsetof(h2s_frames, width), offsetof(h2s_params, pipeline), offsetof(h2s_params, knee_offset),
         offsetof(h2s_params, target_white), offsetof(h2s_params, chroma_edge),
         offsetof(h2s_params, lut_input), offsetof(h2s_params, lp_tone));
  return 0;
}
'''


def test_struct_layout_matches_c(tmp_path):
    c = tmp_path / 'probe.c'
    c.write_text(PROBE)
    exe = tmp_path / 'probe'
    subprocess.run(['gcc', '-I', os.path.dirname(HEADER), str(c), '-o', str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    for P, F in ((_abi.H2SParams, _abi.H2SFrames), (oracle.Params, oracle.Frames)):
        want = [ctypes.sizeof(P), P.tm_param.offset, P.lut_enabled.offset, P.desat_luma.offset,
                ctypes.sizeof(F), F.width.offset, P.pipeline.offset, P.knee_offset.offset,
                P.target_white.offset, P.chroma_edge.offset, P.lut_input.offset, P.lp_tone.offset]
        assert got == want


@pytest.mark.skipif(gpu_available(), reason='checks the no-device error path')
def test_create_without_device_fails_cleanly():
    L = _abi.lib()
    ctx = ctypes.c_void_p()
    rc = L.h2s_create(0, ctypes.byref(ctx))
    assert rc == _abi.H2S_E_HIP and not ctx.value
    assert L.h2s_last_error(None)


def test_null_handling_without_device():
    L = _abi.lib()
    assert L.h2s_set_lut(None, None, 65) == _abi.H2S_E_INVALID_ARG
    assert L.h2s_set_params(None, None) == _abi.H2S_E_INVALID_ARG
    assert L.h2s_process(None, None, None, 1, None) == _abi.H2S_E_INVALID_ARG
    L.h2s_destroy(None)
    assert L.h2s_cube_format(1, None, 0) == _abi.H2S_E_INVALID_ARG
    assert L.h2s_set_option(None, _abi.OPT_FAST_PATH, 0) == _abi.H2S_E_INVALID_ARG
    assert L.h2s_query_path(None, None, None) == _abi.H2S_E_INVALID_ARG
    with pytest.raises(ValueError):
        _abi.raise_for(_abi.H2S_E_UNSUPPORTED, 'x')
    with pytest.raises(FileNotFoundError):
        _abi.raise_for(_abi.H2S_E_LUT_MISSING, 'x')
    with pytest.raises(RuntimeError):
        _abi.raise_for(_abi.H2S_E_HIP, 'x')


def test_product_path_fails_loudly_without_the_library(tmp_path):
    """No CPU fallback: with libh2s missing, the first pixel call raises
    ImportError (the package itself still imports)."""
    import subprocess
    import sys
    code = ('import sys; sys.path.insert(0, %r); import hdr2sdr\n'
            'try:\n    hdr2sdr.Tonemapper(0)\nexcept ImportError as e:\n    print("IMPORTERROR", e)\n'
            'else:\n    print("NO ERROR")\n') % os.path.join(REPO, 'hdr-to-sdr_amd')
    env = dict(os.environ, H2S_LIB=str(tmp_path / 'missing' / 'libh2s.so'))
    out = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=120)
    assert 'IMPORTERROR' in out.stdout, out.stdout + out.stderr


def test_host_package_never_imports_the_oracle():
    """Only tests, smoke() and bench's cpu_baseline may touch oracle/."""
    pkg = os.path.join(REPO, 'hdr-to-sdr_amd', 'hdr2sdr')
    for name in os.listdir(pkg):
        if name.endswith('.py'):
            src = open(os.path.join(pkg, name)).read()
            assert not re.search(r'^\s*(import|from)\s+oracle\b', src, flags=re.M), name


def test_integration_stub_matches_the_abi():
    """INTEGRATION.md's reference-side ctypes stub (the file a maintainer
    adds as src/h2s_backend.py) loads libh2s and mirrors h2s_params /
    h2s_frames field for field (h2s_params_default writes the whole C struct
    into it, so a short mirror would be overwritten past its end)."""
    import re
    doc = open(os.path.join(os.path.dirname(HEADER), '..', 'INTEGRATION.md')).read()
    code = re.search(r'```python\n(# src/h2s_backend.py.*?)```', doc, re.S).group(1)
    env = dict(os.environ, H2S_LIB=_abi.LIB_PATH)
    old = os.environ.get('H2S_LIB')
    os.environ['H2S_LIB'] = env['H2S_LIB']
    try:
        ns = {}
        exec(compile(code, 'INTEGRATION.md', 'exec'), ns)
    finally:
        if old is None:
            del os.environ['H2S_LIB']
        else:
            os.environ['H2S_LIB'] = old
    for mine, ref in ((ns['H2SParams'], _abi.H2SParams), (ns['H2SFrames'], _abi.H2SFrames)):
        assert ctypes.sizeof(mine) == ctypes.sizeof(ref)
        assert [(n, getattr(mine, n).offset) for n, _ in mine._fields_] == \
               [(n, getattr(ref, n).offset) for n, _ in ref._fields_]
