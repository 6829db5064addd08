# kernel trace of the pipelined dynamic-peak schedule (chunk 4): do the
# statistics launches overlap the conversion launches?
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pk_trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pk_trace/raw -o run -- python3 -u scripts/bench_peak_chunk.py 4 > gpurun_out/pk_trace/ab.log 2>&1 || { tail -5 gpurun_out/pk_trace/ab.log; exit 1; }
f=$(find gpurun_out/pk_trace/raw -name "*kernel_trace.csv" | head -1)
python3 - "$f" > gpurun_out/pk_trace/overlap.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the last 40 dispatches (the timed dynamic calls at chunk 4)
tail = rows[-60:]
t0 = int(tail[0]['Start_Timestamp'])
for r in tail:
    print(f"{(int(r['Start_Timestamp'])-t0)/1e3:10.1f} {(int(r['End_Timestamp'])-t0)/1e3:10.1f} q{r.get('Queue_Id','?'):>3} s{r.get('Stream_Id','?'):>3} {r['Kernel_Name'][:60]}")
PY
rm -rf gpurun_out/pk_trace/raw
tail -40 gpurun_out/pk_trace/overlap.txt
