"""scripts/isa_stages.py (the per-stage instruction table of DESIGN.md §4.7)
on a small hand-written listing: stages follow the control-flow graph, not
the text order; an arm of a uniform branch that reaches the join without
the next stage's marker is dropped; the rare region's tone-map markers stay
inside it."""
import importlib.util
import os
import sys

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, 'scripts'))
spec = importlib.util.spec_from_file_location('isa_stages', os.path.join(REPO, 'scripts', 'isa_stages.py'))
st = importlib.util.module_from_spec(spec)
spec.loader.exec_module(st)

LISTING = '''\
k:
\tv_mov_b32 v0, 0
\t;@@body: fast
\t;@@S1 a
\tv_add_f32 v1, v1, v1
\ts_cbranch_vccnz .LBB0_3
; %bb.1:
\tv_mul_f32 v2, v2, v2
\tv_mul_f32 v2, v2, v2
\ts_branch .LBB0_4
.LBB0_3:
\t;@@S2 b
\tv_exp_f32 v3, v3
\tv_fma_f32 v3, v3, v3, v3
.LBB0_4:
\t;@@rare: r
\tv_log_f32 v4, v4
\t;@@S2a inner
\tv_add_f32 v4, v4, v4
\t;@@S3 c
\tv_add_f32 v5, v5, v5
\t;@@tile: store
\tv_add_f32 v6, v6, v6
\ts_endpgm
.Lfunc_end0:
'''


def test_stage_table_follows_the_cfg_and_drops_the_untaken_arm(tmp_path):
    f = tmp_path / 'k.s'
    f.write_text(LISTING)
    blocks = st.parse(str(f), 'k')
    counts, conflicts, entry = st.table(blocks)
    arms, force = st.untaken_arms(blocks, st.successors(blocks), conflicts, entry)
    counts, _, _ = st.table(blocks, arms, force)
    valu = {k[1]: v['valu'] for k, v in counts.items()}
    # %bb.1 (two multiplies) reaches the join still in S1 while the other arm
    # passes S2's marker: it is the untaken arm and is dropped
    assert valu['S1 a'] == 1
    assert valu['S2 b'] == 2 and counts[('fast', 'S2 b')]['trans'] == 1
    # the tone-map marker inside the rare region stays in it
    assert valu['rare: r'] == 1 and valu['rare: r / S2a inner'] == 1
    assert valu['S3 c'] == 1 and valu['tile: store'] == 1
    assert counts[('-', 'tile: store')]['valu'] == 1
