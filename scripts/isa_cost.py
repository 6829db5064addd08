"""Slot-weighted VALU cost of a kernel's basic blocks (static), using the
gfx950 per-opcode throughputs measured by scripts/microbench.hip
(cost relative to v_fma_f32 = 1): full rate for f32 fma/mul/add and integer
add/and/or/mov, 1.65 for max/min/cndmask/cmp/cvt/fract/shift/DPP/VOP3 integer
ops, 3.2 for transcendentals, 1.7 for packed-f32 (2 ops).
Usage: python scripts/isa_cost.py file.s kernel_symbol"""
import re
import sys

FULL = re.compile(r'v_(fma|fmac|fmaak|fmamk|mul|add|sub|subrev)_f32|v_(add|sub|subrev)_u32|v_(and|or|xor)_b32|v_mov_b32_e32|v_mov_b64|v_lshlrev_b16|v_(add|sub)_u16')
TRANS = re.compile(r'v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32')
PK = re.compile(r'v_pk_(fma|mul|add)_f32')


def cost(op):
    if TRANS.match(op):
        return 3.2
    if PK.match(op):
        return 1.7
    if FULL.match(op) and '_dpp' not in op and '_sdwa' not in op:
        return 1.0
    return 1.65


def main():
    path, sym = sys.argv[1], sys.argv[2]
    text = open(path).read().split('\n')
    on = False
    blocks, cur, name = [], [], 'entry'
    for line in text:
        if line.startswith(sym + ':'):
            on = True
            continue
        if not on:
            continue
        if 's_endpgm' in line:
            blocks.append((name, cur))
            break
        m = re.match(r'^(\.LBB\S+):', line)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), []
            continue
        m = re.match(r'\s+(v_\S+)', line)
        if m:
            cur.append(m.group(1))
    tot = 0
    for n, ops in blocks:
        c = sum(cost(o) for o in ops)
        tot += c
        if len(ops) > 20:
            hist = {}
            for o in ops:
                k = o.split('_e32')[0].split('_e64')[0]
                hist[k] = hist.get(k, 0) + cost(o)
            top = sorted(hist.items(), key=lambda kv: -kv[1])[:12]
            print(f'{n:12s} n={len(ops):4d} slots={c:7.1f}  ' + ' '.join(f'{k}:{v:.0f}' for k, v in top))
    print(f'total slots {tot:.1f}')


if __name__ == '__main__':
    main()
