# C3_dyn host round trip: HIP runtime + kernel + memory-copy timeline (no PMC)
set -u
OUT=$PWD/gpurun_out/r04_dyn_rt
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace -d $OUT/trace -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-alt --no-sharded --frames 16 \
  --tonemapper bt.2390 --gamma 1.0 --peak-detect > $OUT/trace.log 2>&1 || { echo trace failed; tail -20 $OUT/trace.log; exit 1; }
ls $OUT/trace
