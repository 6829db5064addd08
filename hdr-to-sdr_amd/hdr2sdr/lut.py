"""The BT.2020->BT.709 3D LUT: generation, .cube text and parsing.

Replaces tools/generate_lut.py (LUT_SIZE = 65, :28; generate_cube_lines,
:93-109) and the bundled asset src/luts/rec2020_to_rec709.cube that
get_lut_filter_path resolves (src/utils.py:212-225).  All arithmetic runs in
libh2s's C++ (h2s_cube_*); this module only moves bytes.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _abi

LUT_SIZE = 65  # tools/generate_lut.py:28
CUBE_NAME = 'rec2020_to_rec709.cube'  # src/utils.py:223


def generate_lattice(size: int = LUT_SIZE) -> np.ndarray:
    """float32 [size^3, 3] in .cube order (red fastest), exactly what lut3d
    holds after parsing the generated file."""
    out = np.empty((size ** 3, 3), dtype=np.float32)
    rc = _abi.lib().h2s_cube_generate(size, out.ctypes.data)
    _abi.raise_for(rc, f'h2s_cube_generate({size})')
    return out


def cube_text(size: int = LUT_SIZE) -> str:
    """Byte-identical to '\\n'.join(generate_cube_lines(size)) + '\\n'."""
    L = _abi.lib()
    n = L.h2s_cube_format(size, None, 0)
    if n < 0:
        _abi.raise_for(int(n), f'h2s_cube_format({size})')
    buf = ctypes.create_string_buffer(n)
    L.h2s_cube_format(size, buf, n)
    return buf.raw[:n].decode('ascii')


def generate_cube_lines(size: int = LUT_SIZE) -> 'list[str]':
    """Same contract as tools/generate_lut.py:93-109."""
    return cube_text(size).rstrip('\n').split('\n')


def parse_cube(text: 'str | bytes') -> np.ndarray:
    """Parse .cube text to float32 [n^3, 3] (.cube order)."""
    data = text.encode('ascii') if isinstance(text, str) else text
    L = _abi.lib()
    n = ctypes.c_int(0)
    rc = L.h2s_cube_parse(data, len(data), None, 0, ctypes.byref(n))
    _abi.raise_for(rc, 'malformed .cube text')
    out = np.empty((n.value ** 3, 3), dtype=np.float32)
    rc = L.h2s_cube_parse(data, len(data), out.ctypes.data, out.size, ctypes.byref(n))
    _abi.raise_for(rc, 'malformed .cube text')
    return out


def escape_path_for_filter(path: str) -> str:
    """src/utils.py:188-204 _escape_path_for_filter: backslashes become '/',
    and the first ':' (the drive colon) becomes two backslashes + ':', as
    ffmpeg's filtergraph parser needs inside lut3d=file=..."""
    return path.replace('\\', '/').replace(':', '\\\\:', 1)


_LUT_FILTER_PATH: 'str | None' = None


def get_lut_filter_path() -> str:
    """src/utils.py:212-225 get_lut_filter_path: the bundled-equivalent
    .cube's path, escaped for direct embedding in the chain string, cached."""
    global _LUT_FILTER_PATH
    if _LUT_FILTER_PATH is None:
        _LUT_FILTER_PATH = escape_path_for_filter(lut_path())
    return _LUT_FILTER_PATH


def unescape_filter_path(path: str) -> str:
    """Inverse of the reference's _escape_path_for_filter (src/utils.py:188-204):
    the drive colon was written as two backslashes + ':' for the filtergraph."""
    return path.replace('\\\\:', ':').replace('\\:', ':')


def load_cube(path: str) -> np.ndarray:
    if not os.path.exists(path):
        # src/utils.py:185-186
        raise FileNotFoundError(f'Required LUT file not found: {path}')
    with open(path, 'rb') as f:
        return parse_cube(f.read())


def lut_path(cache_dir: 'str | None' = None, size: int = LUT_SIZE) -> str:
    """Path of the bundled-equivalent .cube, generating it on first use.

    The reference ships the file (HDR_to_SDR_Converter.spec:29) and treats a
    missing one as a broken install (src/utils.py:212-225); here the file is a
    build artefact of the same generator, written once into ``cache_dir``."""
    d = cache_dir or os.path.join(os.path.dirname(os.path.abspath(__file__)), 'luts')
    os.makedirs(d, exist_ok=True)
    name = CUBE_NAME if size == LUT_SIZE else f'rec2020_to_rec709_{size}.cube'
    p = os.path.join(d, name)
    if not os.path.exists(p):
        tmp = p + f'.tmp{os.getpid()}'
        with open(tmp, 'w', newline='\n') as f:
            f.write(cube_text(size))
        os.replace(tmp, p)
    return p
