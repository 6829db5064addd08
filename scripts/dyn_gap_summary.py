"""The dynamic-peak host round trip, from a rocprofv3 --runtime-trace
--kernel-trace --memory-copy-trace run of `bench.py --peak-detect`: for every
statistics launch, the time from its end to the next tile launch's start, and
what the host spent it on (HIP API calls in between, by name, and the gaps
between them: host compute).  Usage: python scripts/dyn_gap_summary.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(pattern):
    f = glob.glob(os.path.join(sys.argv[1], '**', pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


k = load('*kernel_trace.csv')
api = load('*hip_api_trace.csv')
cp = load('*memory_copy_trace.csv')
kt = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in k)
at = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Function', r.get('Operation', '?'))) for r in api)
ct = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Direction', r.get('Operation', '?'))) for r in cp)
gaps, by = [], defaultdict(list)
for i, (s0, e0, n0) in enumerate(kt):
    if 'k_peak_stats' not in n0:
        continue
    nxt = next(((s, e, n) for s, e, n in kt[i + 1:] if 'k_tile' in n), None)
    if not nxt:
        continue
    gaps.append((nxt[0] - e0) / 1e3)
    for s, e, n in at:
        if e0 <= s < nxt[0]:
            by[n].append((e - s) / 1e3)
    for s, e, n in ct:
        if e0 <= s < nxt[0]:
            by['copy ' + n].append((e - s) / 1e3)
gaps = gaps[2:]   # warm-up
print(f'{len(gaps)} round trips: stats end -> tile start, median {sorted(gaps)[len(gaps) // 2]:.1f} us')
for n, v in sorted(by.items(), key=lambda x: -sum(x[1])):
    print(f'  {n:40s} calls {len(v):4d}  per round trip {sum(v) / max(1, len(gaps) + 2):8.1f} us')
