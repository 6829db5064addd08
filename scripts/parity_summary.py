"""Summarise a parity report (H2S_PARITY_REPORT, written by the -m gpu suite's
integer checks) as the markdown tables DESIGN.md §2 carries.

Usage: python scripts/parity_summary.py profiles/r04/parity_report.jsonl
"""
import json
import sys
from collections import defaultdict


def pct(x: float) -> str:
    return f'{100 * x:.3f} %'


def main(path: str) -> None:
    rows = [json.loads(line) for line in open(path) if line.strip()]
    print(f'{len(rows)} integer checks\n')
    print('| check | size | quantiser | luma exact / 1 step / beyond | chroma exact / 1 step / beyond | max diff (output steps) |')
    print('|---|---|---|---|---|---|')
    for r in rows:
        if 'test_00_gpu_baseline' not in r['test']:
            continue
        name = r['test'].split('::')[1]
        lu, ch = r['luma'], r['chroma']
        print(f"| {name} | {r['W']}x{r['H']}x{r['frames']} | {r['quantiser_bits']} | "
              f"{pct(lu['exact'])} / {pct(lu['one_step'])} / {pct(lu['beyond'])} | "
              f"{pct(ch['exact'])} / {pct(ch['one_step'])} / {pct(ch['beyond'])} | {r['max_diff_out_steps']} |")
    agg = defaultdict(lambda: {'n': 0, 'min_exact': 1.0, 'max_beyond': 0.0, 'max_steps': 0, 'worst': ''})
    for r in rows:
        a = agg[r['pipeline']]
        a['n'] += 1
        ex = min(r['luma']['exact'], r['chroma']['exact'])
        if ex < a['min_exact']:
            a['min_exact'], a['worst'] = ex, r['test'].split('::')[1]
        a['max_beyond'] = max(a['max_beyond'], r['luma']['beyond'], r['chroma']['beyond'])
        a['max_steps'] = max(a['max_steps'], r['max_diff_out_steps'])
    print('\n| pipeline | checks | lowest exact share (where) | largest beyond-one-step share | largest diff (output steps) |')
    print('|---|---|---|---|---|')
    for k, a in sorted(agg.items()):
        print(f"| {k} | {a['n']} | {pct(a['min_exact'])} ({a['worst']}) | {pct(a['max_beyond'])} | {a['max_steps']} |")


if __name__ == '__main__':
    main(sys.argv[1])
