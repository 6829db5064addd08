"""LUT lattice parity: oracle restatement and product generator vs the
reference's own tools/generate_lut.py output (golden hashes captured by
tests/golden/make_golden.py).  Mirrors test/generator_drift_test.py:20-34."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import hdr2sdr


@pytest.fixture(scope='module')
def hashes(golden_dir):
    with open(os.path.join(golden_dir, 'lut_hashes.json')) as f:
        return json.load(f)['sizes']


@pytest.mark.parametrize('n', [2, 3, 17, 33, 65])
def test_oracle_generator_matches_reference_bytes(hashes, n):
    text = ('\n'.join(oracle.generate_cube_lines(n)) + '\n').encode()
    assert hashlib.sha256(text).hexdigest() == hashes[str(n)]['sha256']
    assert len(text) == hashes[str(n)]['bytes']


@pytest.mark.parametrize('n', [2, 3, 17, 33, 65])
def test_product_generator_matches_reference_bytes(hashes, n):
    text = hdr2sdr.cube_text(n).encode()
    assert hashlib.sha256(text).hexdigest() == hashes[str(n)]['sha256']
    assert hashlib.md5(text).hexdigest() == hashes[str(n)]['md5']


@pytest.mark.parametrize('n', [17, 65])
def test_sampled_rows_and_header(hashes, n):
    lines = hdr2sdr.generate_cube_lines(n)
    g = hashes[str(n)]
    assert lines[0] == g['header'] == f'LUT_3D_SIZE {n}'
    for i, row in g['rows'].items():
        assert lines[1 + int(i)] == row


def test_convert_matches_reference_points(golden_dir):
    with open(os.path.join(golden_dir, 'lut_convert.json')) as f:
        pts = json.load(f)['points']
    for p in pts:
        assert list(oracle.convert(*p['in'])) == p['out']   # bit-exact doubles


def test_lattice_is_parsed_text(hashes):
    """h2s_cube_generate == parse(h2s_cube_format) == oracle parse (float32,
    decimal -> double -> float as lut3d)."""
    for n in (17, 65):
        lat = hdr2sdr.generate_lattice(n)
        assert lat.shape == (n ** 3, 3) and lat.dtype == np.float32
        assert np.array_equal(lat, hdr2sdr.parse_cube(hdr2sdr.cube_text(n)))
        assert np.array_equal(lat, oracle.parse_cube(hdr2sdr.cube_text(n)))


def test_lattice_properties():
    lat = hdr2sdr.generate_lattice(65).reshape(65, 65, 65, 3)  # [b, g, r, c]
    assert lat.min() >= 0 and lat.max() <= 1
    # neutral axis stays neutral (matrix rows sum to 1)
    d = np.arange(65)
    grey = lat[d, d, d]
    assert np.abs(grey - grey[:, :1]).max() <= 1e-6
    # corners: black, white
    assert np.array_equal(lat[0, 0, 0], [0, 0, 0])
    assert np.allclose(lat[64, 64, 64], [1, 1, 1], atol=1e-6)


def test_parse_cube_edge_cases():
    txt = '# comment\nTITLE "x"\nDOMAIN_MIN 0 0 0\nDOMAIN_MAX 1 1 1\nLUT_3D_SIZE 2\n' + \
          '\n'.join(f'{i / 8:.6f} 0.5 0.25' for i in range(8)) + '\n'
    a = hdr2sdr.parse_cube(txt)
    assert a.shape == (8, 3) and a[3, 0] == np.float32(0.375)
    with pytest.raises(ValueError):
        hdr2sdr.parse_cube('LUT_3D_SIZE 2\n0 0 0\n')            # too few rows
    with pytest.raises(ValueError):
        hdr2sdr.parse_cube('0 0 0\n')                            # no header
    with pytest.raises(ValueError):
        hdr2sdr.parse_cube('DOMAIN_MAX 2 2 2\nLUT_3D_SIZE 2\n' + '0 0 0\n' * 8)  # unsupported domain
    with pytest.raises(ValueError):
        hdr2sdr.parse_cube('LUT_1D_SIZE 4\n')


def test_lut_path_generates_once(tmp_path, hashes):
    from hdr2sdr import lut
    p = lut.lut_path(str(tmp_path), size=17)
    with open(p, 'rb') as f:
        assert hashlib.sha256(f.read()).hexdigest() == hashes['17']['sha256']
    m = os.path.getmtime(p)
    assert lut.lut_path(str(tmp_path), size=17) == p and os.path.getmtime(p) == m
    with pytest.raises(FileNotFoundError):
        lut.load_cube(str(tmp_path / 'missing.cube'))


@pytest.mark.parametrize('raw,esc', [
    (r'C:\Program Files\HDR\luts\rec2020_to_rec709.cube', r'C\\:/Program Files/HDR/luts/rec2020_to_rec709.cube'),
    ('/opt/app/luts/rec2020_to_rec709.cube', '/opt/app/luts/rec2020_to_rec709.cube'),
    (r'D:\a:b.cube', r'D\\:/a:b.cube'),      # only the first colon is escaped
])
def test_escape_path_for_filter_matches_reference_rule(raw, esc):
    from hdr2sdr.lut import escape_path_for_filter, unescape_filter_path
    assert escape_path_for_filter(raw) == esc
    assert unescape_filter_path(esc) == raw.replace('\\', '/')


def test_get_lut_filter_path_points_at_the_generated_cube():
    from hdr2sdr.lut import get_lut_filter_path, unescape_filter_path, load_cube, generate_lattice
    p = unescape_filter_path(get_lut_filter_path())
    assert np.array_equal(load_cube(p), generate_lattice(65))
