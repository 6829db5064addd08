set -u -o pipefail
mkdir -p gpurun_out/r05_bench_dyn
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_dyn/bench.log 2>&1 || { tail -5 gpurun_out/r05_bench_dyn/bench.log; exit 1; }
tail -1 gpurun_out/r05_bench_dyn/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['other_configs']['C3_dyn'], d['config']['other_configs']['C3']['kernel_ms'])"
