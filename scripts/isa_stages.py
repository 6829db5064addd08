"""Per-stage instruction and slot table of one k_tile instance, from an ISA
listing built with -DH2S_ISA_MARKS (h2s_tile.h H2S_MARK: each marker is an
assembler comment ";@@name" that opens stage `name`).

The listing's basic blocks are laid out by the compiler, not in source
order, so a block's stage is not the last marker above it in the text: the
stage flows along the control-flow graph (branch targets and fall-through)
from the marker that opened it.  Markers "body: fast" / "body: exact-capable"
name which of the two step bodies (h2s_tile.h steps<FB>) a stage belongs to;
"tile: ..." markers are per-tile work (8 steps of one wave per tile), and
"rare: ..." stages (the dark re-run) are taken by ~1 % of the steps and are
listed apart.

A uniform branch (a launch- or block-uniform flag, e.g. libplacebo's black
point lift with bp = 4 or not) leaves both arms in the listing; --skip BLOCK
drops arms the measured workload never takes, by label.

Per pixel: one step is 64 pixels, one per lane, so a step body's wave
instructions / 8 unrolled steps = instructions per pixel; a tile's work is
shared by its 8 steps per wave.  Slots weight each VALU opcode by its gfx950
issue cost (scripts/isa_cost.py).

Usage: python scripts/isa_stages.py listing.s kernel_symbol [--body fast]
       [--skip .LBB0_12,...]"""
import argparse
import re
from collections import OrderedDict, defaultdict, deque

from isa_cost import cost

LABEL = re.compile(r'^(\.LBB\d+_\d+):|^; (%bb\.\d+):')   # (fall-through-only blocks are comments)
MARK = re.compile(r';@@(.*)$')
INSN = re.compile(r'^\s+([a-z_][a-z0-9_]*)\b(.*)$')


def parse(path, sym):
    """-> [(label, [items])], items ('mark', name) or ('insn', op, operands)."""
    blocks, cur, name, on = [], [], 'entry', False
    for line in open(path):
        line = line.rstrip('\n')
        if not on:
            on = line.startswith(sym + ':')
            continue
        if line.startswith('.Lfunc_end'):
            break
        m = LABEL.match(line)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1) or m.group(2), []
            continue
        m = MARK.search(line)
        if m:
            cur.append(('mark', m.group(1).strip()))
            continue
        m = INSN.match(line)
        if m and not m.group(1).startswith('.'):
            cur.append(('insn', m.group(1), m.group(2)))
    blocks.append((name, cur))
    return [(n, it) for n, it in blocks if it or n != 'entry']


def successors(blocks):
    idx = {n: i for i, (n, _) in enumerate(blocks)}
    succ = []
    for i, (n, items) in enumerate(blocks):
        ins = [it for it in items if it[0] == 'insn']
        last = ins[-1] if ins else None
        # a block may end in two terminators: s_cbranch_* A; s_branch B
        s = [idx[it[2].strip().split()[0]] for it in ins if it[1].startswith('s_cbranch')]
        if last and last[1] == 's_branch':
            s.append(idx[last[2].strip().split()[0]])
        elif not (last and last[1] in ('s_endpgm', 's_setpc_b64')) and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    return succ


def step(state, mark):
    """The stage a marker opens.  Inside a rare region (the dark re-run calls
    the tone map again), the tone map's own markers (S2a..S2c) stay in it;
    the next marker of the chain ends it."""
    body, stage = state
    if mark.startswith('body: '):
        return (mark[6:], 'set-up')
    if mark.startswith('tile: '):
        return ('-', mark)
    if stage.startswith('rare') and re.match(r'S2[a-c] ', mark):
        return (body, stage.split(' / ')[0] + ' / ' + mark)
    return (body, mark)


def classify(op):
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('buffer_', 'global_', 'flat_')):
        return 'vmem'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def untaken_arms(blocks, succ, conflicts, entry):
    """A launch-uniform branch (lp_ipt, lut_off, ...) joins two arms: the
    one the instance's own workload takes passes the next stage's marker (the
    IPT form's S2a..S2c, the lut3d table's S4 / S5); the other carries none
    and reaches the join in the earlier stage.  -> (blocks of the marker-less
    arms, {join: the later stage})."""
    def marked(i):
        return any(it[0] == 'mark' for it in blocks[i][1])
    skip, force = set(), {}
    for j, s1, s2 in conflicts:
        if s1[0] != s2[0] or not (s1[1].startswith('S') and s2[1].startswith('S')):
            continue   # (the tile loop's back edge, not an arm)
        late, early = (s1, s2) if s1[1] > s2[1] else (s2, s1)
        force[j] = late
        arm = {i for i in range(len(blocks)) if j in succ[i] and not marked(i) and entry[i] == early}
        grow = True
        while grow:
            grow = False
            for i in range(len(blocks)):
                if i in arm or marked(i) or entry[i] != early or not succ[i]:
                    continue
                if all(k in arm or k == j for k in succ[i]):
                    arm.add(i)
                    grow = True
        skip |= arm
    return skip, force


def table(blocks, skip=(), force=None):
    succ = successors(blocks)
    entry_state = [None] * len(blocks)
    entry_state[0] = ('-', 'prologue')
    force = force or {}
    for j, st in force.items():
        entry_state[j] = st
    conflicts = []
    q = deque([0])
    counts = defaultdict(lambda: defaultdict(float))
    done = set()
    while q:
        i = q.popleft()
        if i in done:
            continue
        done.add(i)
        name, items = blocks[i]
        st = entry_state[i]
        counted = name not in skip and i not in skip
        for it in items:
            if it[0] == 'mark':
                st = step(st, it[1])
                continue
            if not counted:
                continue
            c = counts[st]
            k = classify(it[1])
            c[k] += 1
            if k == 'valu':
                c['op:' + it[1].split('_e32')[0].split('_e64')[0]] += 1
            if k == 'valu':
                c['slots'] += cost(it[1])
                if re.match(r'v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32', it[1]):
                    c['trans'] += 1
        for j in succ[i]:
            if j in force and j not in done:
                q.append(j)
            elif entry_state[j] is None:
                entry_state[j] = st
                q.append(j)
            elif entry_state[j] != st and blocks[j][0] not in skip and i not in skip and j not in force:
                conflicts.append((j, entry_state[j], st))
    return counts, conflicts, entry_state


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('listing')
    ap.add_argument('symbol')
    ap.add_argument('--body', default='fast')
    ap.add_argument('--skip', default='')
    ap.add_argument('--steps', type=int, default=8)
    ap.add_argument('--ops', default='', help='print the VALU opcode histogram of the stages containing this text')
    a = ap.parse_args()
    blocks = parse(a.listing, a.symbol)
    skip = set(filter(None, a.skip.split(',')))
    counts, conflicts, entry = table(blocks, skip)
    # second pass: the arms the instance's workload does not take dropped
    arms, force = untaken_arms(blocks, successors(blocks), conflicts, entry)
    counts, conflicts, _ = table(blocks, skip | arms, force)
    rows = OrderedDict()
    for (body, stage), c in counts.items():
        if body in (a.body, '-'):
            rows[(body, stage)] = c
    print(f'| stage ({a.body} body) | VALU / px | of which transcendental | slots / px | LDS / px | vector memory / px | SALU / px |')
    print('|---|---|---|---|---|---|---|')
    tot = defaultdict(float)
    for (body, stage), c in sorted(rows.items(), key=lambda kv: kv[0][1]):
        if stage == 'prologue':
            continue
        d = a.steps
        line = f"| {stage} | {c['valu'] / d:.1f} | " \
               f"{c['trans'] / d:.1f} | {c['slots'] / d:.1f} | {c['lds'] / d:.2f} | {c['vmem'] / d:.2f} | {c['salu'] / d:.1f} |"
        print(line)
        if not stage.startswith('rare'):
            for k in ('valu', 'trans', 'slots', 'lds', 'vmem', 'salu'):
                tot[k] += c[k] / d
    print(f"| **total (without rare)** | **{tot['valu']:.1f}** | {tot['trans']:.1f} | **{tot['slots']:.1f}** | "
          f"{tot['lds']:.2f} | {tot['vmem']:.2f} | {tot['salu']:.1f} |")
    if a.ops:
        for (body, stage), c in rows.items():
            if a.ops in stage:
                ops = sorted(((v, k[3:]) for k, v in c.items() if k.startswith('op:')), reverse=True)
                print(f'\n{stage}: ' + ', '.join(f'{k} {v / a.steps:.2f}' for v, k in ops))
    # joins after the rare re-run and the tile loop's back edge are expected;
    # anything else means a stage boundary the markers do not resolve
    odd = [c for c in conflicts if not any(x[1].startswith(('S', 'rare', 'prologue', 'tile')) for x in c[1:])]
    for j, s1, s2 in odd[:20]:
        print('unresolved join', blocks[j][0], s1, s2)


if __name__ == '__main__':
    main()
