"""The in-tree build (hdr2sdr/_build.py): the gpurun snapshot carries
libh2s.so and its flag stamp but not the objects (build/ is gpurun-ignored),
so a current library must not be recompiled on the GPU box; a flag change
still rebuilds."""
import pytest

from hdr2sdr import _build


class _Compiled(Exception):
    pass


def _no_compiler(*a, **k):
    raise _Compiled(a[0] if a else k)


def test_a_current_library_without_its_objects_is_not_rebuilt(tmp_path, monkeypatch):
    monkeypatch.setattr(_build, 'OBJ_DIR', str(tmp_path / 'obj'))
    monkeypatch.setattr(_build.subprocess, 'run', _no_compiler)
    assert _build.build_lib() == _build.LIB


def test_a_flag_change_rebuilds(tmp_path, monkeypatch):
    monkeypatch.setattr(_build, 'OBJ_DIR', str(tmp_path / 'obj'))
    monkeypatch.setattr(_build.subprocess, 'run', _no_compiler)
    monkeypatch.setattr(_build, '_hipcc', lambda: 'hipcc')
    monkeypatch.setattr(_build, 'CFLAGS', _build.CFLAGS + ['-DH2S_FLAG_CHANGED'])
    with pytest.raises(_Compiled):
        _build.build_lib()
