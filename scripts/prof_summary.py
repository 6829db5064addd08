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


def unit_shares(m):
    """What binds the kernel, from per-dispatch counter
    means m.  GRBM_GUI_ACTIVE is summed over the 8 XCDs (32 CUs each).
    - valu_insts_per_cu_cycle: SQ_INSTS_VALU / (cycles x 256), the figure
      VERDICT r04 defined;
    - valu_issue_frac: the same against the CU's VALU rate on gfx950 -- four
      SIMD-32 units, a wave64 full-rate op 2 cycles, a transcendental 4
      (MI355X_MICROARCH.md, constants table: v_fma 2 cyc; issue cost of one
      wave alone v_exp 8 vs v_fma 4) -- i.e. (VALU + TRANS) / (cycles x 512).
      1.0 is the ceiling; the C3 instance measures 1.12-1.15 VALU wave-
      instructions per CU-cycle, so one per cycle is not.  Every other VALU
      op counts at the full rate (a lower bound: compares, selects,
      conversions, min/max and DPP measured ~1.65x);
    - valu_waves_per_simd: SQ_ACTIVE_INST_VALU (quad-cycles, counted per
      wave and summed over waves) per SIMD-cycle: the mean number of a
      SIMD's waves that have a VALU instruction in flight.  It is an
      occupancy, not a fraction (two waves overlapping on one SIMD count
      twice), so it may pass 1; until round 6 it was reported as
      'valu_active_frac' (VERDICT r05 item 2).  The VALU's utilisation is
      valu_issue_frac;
    - td_busy_frac / td_tc_stall_frac / ta_busy_frac: the texture data unit
      (L1 -> VGPR return, one per CU) busy, and the share of it waiting for
      the L1; the texture address unit."""
    out = {}
    if 'GRBM_GUI_ACTIVE' not in m:
        return out
    cyc = m['GRBM_GUI_ACTIVE'] / 8.0
    out['cycles_per_dispatch'] = round(cyc)
    if 'SQ_INSTS_VALU' in m:
        out['valu_insts_per_cu_cycle'] = round(m['SQ_INSTS_VALU'] / (cyc * 256), 4)
        out['valu_issue_frac'] = round((m['SQ_INSTS_VALU'] + m.get('SQ_INSTS_VALU_TRANS_F32', 0.0))
                                       / (cyc * 512), 4)
    if 'SQ_ACTIVE_INST_VALU' in m:
        out['valu_waves_per_simd'] = round(4 * m['SQ_ACTIVE_INST_VALU'] / (cyc * 1024), 4)
    for key, ctr in (('td_busy_frac', 'TD_TD_BUSY_sum'), ('td_tc_stall_frac', 'TD_TC_STALL_sum'),
                     ('ta_busy_frac', 'TA_TA_BUSY_sum')):
        if ctr in m:
            out[key] = round(m[ctr] / (cyc * 256), 4)
    return out


def from_summary(d):
    """Re-derive the unit shares of an existing traffic.json from the counter
    means its summary.txt lists (for runs whose raw CSVs were not kept)."""
    m = {}
    for line in open(os.path.join(d, 'summary.txt')):
        parts = line.split()
        if len(parts) == 3 and parts[2].startswith('(n=') and parts[0][:1].isupper():
            m[parts[0]] = float(parts[1])
    path = os.path.join(d, 'traffic.json')
    rec = json.load(open(path))
    for k in ('valu_issue_frac', 'valu_active_frac', 'valu_waves_per_simd', 'td_busy_frac',
              'cycles_per_dispatch'):
        rec.pop(k, None)
    rec.update(unit_shares(m))
    with open(path, 'w') as f:
        json.dump(rec, f, indent=1)
    print('traffic.json:', json.dumps(rec))


def main(d):
    """Summarise profile directory d; write d/traffic.json."""
    # the C2 instance k_tile<PQ, Hable, RGB desat, CPU chain, DBG 0>
    KERNEL = os.environ.get('H2S_PROF_KERNEL', 'k_tile<0, 5, 2, 0, 0>')   # (H2S_PROF_KERNEL: another instance)

    for f in glob.glob(os.path.join(d, 'trace', '**', '*kernel_stats.csv'), recursive=True):
        print('## kernel stats', os.path.relpath(f, d))
        for row in csv.DictReader(open(f)):
            if KERNEL in row['Name']:
                print(f"{row['Name'][:60]}: calls={row['Calls']} avg_ns={float(row['AverageNs']):.0f} "
                      f"min_ns={row['MinNs']} max_ns={row['MaxNs']}")
    # the warm average: the trace run's dispatches of the kernel after its
    # warm-up (the bench's --warmup launches, from the trace log's own line)
    for f in glob.glob(os.path.join(d, 'trace', '**', '*kernel_trace.csv'), recursive=True):
        dur = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) for r in csv.DictReader(open(f))
               if KERNEL in r['Kernel_Name']]
        warm, bench_ms = None, None
        log = os.path.join(d, 'trace.log')
        if os.path.exists(log):
            for line in open(log):
                if line.startswith('{'):
                    rec = json.loads(line)
                    warm, bench_ms = rec.get('warmup'), rec.get('roofline', {}).get('kernel_ms')
                    step_ms, steps = rec.get('ms_per_step'), rec.get('steps')
        if dur and warm is not None and len(dur) >= warm + steps:
            w = dur[warm:warm + steps]   # the timed launches of the headline run
            print(f'## warm kernel trace: the {len(w)} timed dispatches after {warm} warm-up ones: avg_ns={sum(w) / len(w):.0f} '
                  f'median_ns={sorted(w)[len(w) // 2]} min_ns={min(w)}; the same run\'s HIP-event kernel_ms '
                  f'{bench_ms} and ms_per_step {step_ms}')

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
        rec.update(unit_shares({k: sum(v) / len(v) for k, v in vals.items()}))
        with open(os.path.join(d, 'traffic.json'), 'w') as f:
            json.dump(rec, f, indent=1)
        print('traffic.json:', json.dumps(rec))


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--from-summary':
        from_summary(sys.argv[2])
    else:
        main(sys.argv[1])
