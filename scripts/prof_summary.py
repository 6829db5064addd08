"""Summarise a scripts/profile.sh directory: per-kernel average duration from
the kernel-trace stats and per-dispatch averages of every PMC counter for
k_tile, with the gfx950 FETCH_SIZE correction (x2 for wide coalesced
streaming reads, MI355X_MICROARCH.md §HBM).  Also writes traffic.json (HBM
bytes per dispatch + the bench workload it was measured on), which bench.py
reports as roofline.traffic when its own workload matches."""
import csv
import json
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
# the C2 instance k_tile<PQ, Hable, RGB desat, CPU chain, DBG 0>
KERNEL = os.environ.get('H2S_PROF_KERNEL', 'k_tile<0, 5, 2, 0, 0>')   # (H2S_PROF_KERNEL: another instance)

for f in glob.glob(os.path.join(d, 'trace', '**', '*kernel_stats.csv'), recursive=True):
    print('## kernel stats', os.path.relpath(f, d))
    for row in csv.DictReader(open(f)):
        if KERNEL in row['Name']:
            print(f"{row['Name'][:60]}: calls={row['Calls']} avg_ns={float(row['AverageNs']):.0f} "
                  f"min_ns={row['MinNs']} max_ns={row['MaxNs']}")

vals = defaultdict(list)
for f in glob.glob(os.path.join(d, 'pmc_*', '**', '*counter_collection.csv'), recursive=True):
    for row in csv.DictReader(open(f)):
        if KERNEL not in row.get('Kernel_Name', ''):
            continue
        vals[row['Counter_Name']].append(float(row['Counter_Value']))
print('## PMC per k_tile dispatch (mean over dispatches)')
for k in sorted(vals):
    v = vals[k]
    print(f'{k:28s} {sum(v) / len(v):18.1f}   (n={len(v)})')
if 'FETCH_SIZE' in vals:
    fs = sum(vals['FETCH_SIZE']) / len(vals['FETCH_SIZE'])
    print(f'FETCH_SIZE corrected (x2, KiB->B): {fs * 2 * 1024:.0f} B per dispatch')
if 'WRITE_SIZE' in vals:
    ws = sum(vals['WRITE_SIZE']) / len(vals['WRITE_SIZE'])
    print(f'WRITE_SIZE (KiB->B): {ws * 1024:.0f} B per dispatch')

if 'FETCH_SIZE' in vals and 'WRITE_SIZE' in vals:
    workload = None
    log = os.path.join(d, 'pmc_fetch.log')
    if os.path.exists(log):
        for line in open(log):
            if line.startswith('{'):
                workload = json.loads(line)['config']['workload']
    rec = {'kernel': KERNEL, 'workload': workload,
           'fetch_bytes_per_dispatch': int(fs * 2 * 1024), 'write_bytes_per_dispatch': int(ws * 1024),
           'bytes_per_dispatch': int(fs * 2 * 1024 + ws * 1024),
           'method': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950), KiB->B',
           'dispatches': len(vals['FETCH_SIZE'])}
    # instruction mix per pixel (wave instructions x 64 lanes / pixels of one dispatch)
    px = None
    if workload:
        import re
        m = re.search(r'(\d+)x(\d+) .*?(\d+) frames per launch', workload)
        if m:
            px = int(m.group(1)) * int(m.group(2)) * int(m.group(3))
    if px:
        for key, ctr in (('valu_per_px', 'SQ_INSTS_VALU'), ('trans_per_px', 'SQ_INSTS_VALU_TRANS_F32'),
                         ('cvt_per_px', 'SQ_INSTS_VALU_CVT'), ('lds_per_px', 'SQ_INSTS_LDS'),
                         ('vmem_rd_per_px', 'SQ_INSTS_VMEM_RD')):
            if ctr in vals:
                rec[key] = round(sum(vals[ctr]) / len(vals[ctr]) * 64 / px, 2)
    # what binds the kernel: VALU wave-instructions
    # issued per CU-cycle (one per cycle is the 4 SIMDs' peak for wave64 full-
    # rate ops), the texture-data unit's busy share, per the cycles of the
    # dispatch (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 32 CUs each)
    if 'GRBM_GUI_ACTIVE' in vals:
        cyc = sum(vals['GRBM_GUI_ACTIVE']) / len(vals['GRBM_GUI_ACTIVE']) / 8.0
        rec['cycles_per_dispatch'] = round(cyc)
        if 'SQ_INSTS_VALU' in vals:
            rec['valu_issue_frac'] = round(sum(vals['SQ_INSTS_VALU']) / len(vals['SQ_INSTS_VALU']) / (cyc * 256), 4)
        if 'SQ_ACTIVE_INST_VALU' in vals:
            rec['valu_active_frac'] = round(4 * sum(vals['SQ_ACTIVE_INST_VALU']) / len(vals['SQ_ACTIVE_INST_VALU'])
                                            / (cyc * 1024), 4)
        if 'TD_TD_BUSY_sum' in vals:
            rec['td_busy_frac'] = round(sum(vals['TD_TD_BUSY_sum']) / len(vals['TD_TD_BUSY_sum']) / (cyc * 256), 4)
    with open(os.path.join(d, 'traffic.json'), 'w') as f:
        json.dump(rec, f, indent=1)
    print('traffic.json:', json.dumps(rec))
