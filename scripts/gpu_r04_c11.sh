# C3 with peak_detect=1 (C3_dyn): per-kernel time of the statistics launch
# against the tile launch (histogram LDS atomics)
set -u
OUT=$PWD/gpurun_out/r04_dyn
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-alt --no-sharded --frames 16 \
  --tonemapper bt.2390 --gamma 1.0 --peak-detect > $OUT/trace.log 2>&1 || { echo trace failed; tail -20 $OUT/trace.log; exit 1; }
cat $OUT/trace/run_kernel_stats.csv | cut -c1-200
