"""Average duration per (kernel, grid) from a rocprofv3 kernel-trace CSV
(several launch shapes of one kernel in one run: the A/B sweeps of
scripts/bench_peak_stats.py).  Usage: python scripts/trace_by_grid.py TRACE.csv [substring...]"""
import csv
import sys
from collections import defaultdict

rows = defaultdict(list)
with open(sys.argv[1]) as fh:
    for r in csv.DictReader(fh):
        name = r['Kernel_Name']
        if len(sys.argv) > 2 and not any(s in name for s in sys.argv[2:]):
            continue
        key = (name[:70], r['Grid_Size_X'], r['Grid_Size_Y'], r['VGPR_Count'])
        rows[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000.0)
for (name, gx, gy, vg), d in sorted(rows.items()):
    d.sort()
    print(f'{name:70s} grid {gx:>7s} x {gy:>3s} vgpr {vg:>3s}  n {len(d):4d}  avg {sum(d) / len(d):8.2f} us  '
          f'median {d[len(d) // 2]:8.2f}  min {d[0]:8.2f}')
