set -u -o pipefail
mkdir -p gpurun_out/r05_tpb_small
timeout -k 10 300 python -u scripts/bench_tpb_small.py > gpurun_out/r05_tpb_small/tpb.log 2>&1 || { tail -5 gpurun_out/r05_tpb_small/tpb.log; exit 1; }
tail -1 gpurun_out/r05_tpb_small/tpb.log
