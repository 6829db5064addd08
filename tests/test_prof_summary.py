"""The PMC post-processing behind bench.py's roofline (CPU): the unit shares
scripts/prof_summary.py derives from the counter means,
the committed closing profiles re-derived from their own summaries, and the
bench's traffic lookup by workload string."""
import importlib.util
import json
import os
import shutil

import pytest

from conftest import REPO


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ps = _load('prof_summary', os.path.join(REPO, 'scripts', 'prof_summary.py'))


def test_unit_shares_formulas():
    cyc = 1000.0
    m = {'GRBM_GUI_ACTIVE': 8 * cyc,                  # summed over the 8 XCDs
         'SQ_INSTS_VALU': 0.9 * 256 * cyc, 'SQ_INSTS_VALU_TRANS_F32': 0.1 * 256 * cyc,
         'SQ_ACTIVE_INST_VALU': 0.25 * 1024 * cyc,    # quad-cycles
         'TD_TD_BUSY_sum': 0.93 * 256 * cyc, 'TD_TC_STALL_sum': 0.5 * 256 * cyc, 'TA_TA_BUSY_sum': 0.7 * 256 * cyc}
    u = ps.unit_shares(m)
    assert u['cycles_per_dispatch'] == 1000
    assert u['valu_insts_per_cu_cycle'] == pytest.approx(0.9)
    # gfx950: a wave64 full-rate op takes 2 cycles of a SIMD-32, a
    # transcendental 4: 2 wave-instructions per CU-cycle is the ceiling
    assert u['valu_issue_frac'] == pytest.approx((0.9 + 0.1) / 2)
    # waves with a VALU instruction in flight per SIMD: an occupancy, not a
    # fraction of the issue rate
    assert u['valu_waves_per_simd'] == pytest.approx(1.0) and 'valu_active_frac' not in u
    assert (u['td_busy_frac'], u['td_tc_stall_frac'], u['ta_busy_frac']) == pytest.approx((0.93, 0.5, 0.7))
    assert ps.unit_shares({}) == {}


@pytest.mark.parametrize('sub', ['r05/closing/prof', 'r05/closing/prof_c3', 'r06/closing/prof_c2', 'r06/closing/prof_c3'])
def test_closing_profiles_rederive_from_their_summaries(tmp_path, sub):
    """profiles/<round>/closing/<sub>/traffic.json holds what its
    summary.txt's counter means give (the raw per-dispatch CSVs are not kept)."""
    src = os.path.join(REPO, 'profiles', *sub.split('/'))
    for f in ('summary.txt', 'traffic.json'):
        shutil.copy(os.path.join(src, f), tmp_path / f)
    ps.from_summary(str(tmp_path))
    want = json.load(open(os.path.join(src, 'traffic.json')))
    got = json.load(open(tmp_path / 'traffic.json'))
    assert got == want
    assert got['valu_issue_frac'] < 1.0 < got['valu_insts_per_cu_cycle'] * 2


def test_bench_reads_the_c2_traffic_of_its_own_workload():
    """The newest round's profile of the bench's own workload wins
    (profiles/r06/traffic.json: the round-6 closing profile of C2)."""
    bench = _load('bench_mod', os.path.join(REPO, 'bench.py'))
    c2 = json.load(open(os.path.join(REPO, 'profiles', 'r06', 'traffic.json')))
    tr = bench.pmc_traffic(c2['workload'])
    assert tr is not None and tr['source'].startswith('profiles/r06/traffic.json')
    assert tr['bytes_per_dispatch'] == c2['bytes_per_dispatch']
    assert bench.pmc_traffic(c2['workload'].replace('64 frames', '16 frames')) is None
