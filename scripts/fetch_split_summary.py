"""Summarise scripts/prof_fetch_split.sh: per config, k_tile's FETCH_SIZE
(x2, KiB -> B, the gfx950 correction for 128-B streaming requests) and
WRITE_SIZE per dispatch with the 65^3 and the 2^3 lattice."""
import csv
import glob
import os
import sys

out = sys.argv[1]
B_ALG_IN = 64 * 3840 * 2160 * 3     # 10-bit 4:2:0 input bytes per 64-frame launch
rows = {}
for d in sorted(glob.glob(os.path.join(out, '*_lut*_*SIZE'))):
    tag = os.path.basename(d)
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        continue
    vals = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if 'k_tile' in r.get('Kernel_Name', '') and r.get('Counter_Name') in ('FETCH_SIZE', 'WRITE_SIZE'):
                    vals.append(float(r['Counter_Value']))
    if vals:
        vals.sort()
        rows[tag] = vals[len(vals) // 2] * 1024   # median dispatch, KiB -> B
libs = sorted({t.split('.')[0] for t in rows if '.' in t}) or ['']
for lib in libs:
  pre = f'{lib}.' if lib else ''
  for cfg in ('c2', 'c3', 'c3cpu', 'c3max', 'c3hable', 'c2web', 'c3web'):
    f65, f2 = rows.get(f'{pre}{cfg}_lut65_FETCH_SIZE'), rows.get(f'{pre}{cfg}_lut2_FETCH_SIZE')
    w65 = rows.get(f'{pre}{cfg}_lut65_WRITE_SIZE')
    if f65 is None or f2 is None:
        continue
    w65 = w65 or 0.0
    print(f'{pre}{cfg}: FETCH raw 65^3 {f65:.4g} B, 2^3 {f2:.4g} B, lattice-induced {f65 - f2:.4g} B raw '
          f'({(f65 - f2) / B_ALG_IN:.3f} x input); x2-corrected totals {2 * f65:.4g} / {2 * f2:.4g} '
          f'(input {B_ALG_IN:.4g}); WRITE {w65:.4g} B')
