# round-4 closing evidence, part A: the -m gpu suite (parity + float reports),
# the default bench line, smoke()
set -u
PYTEST_STOP=--maxfail=20 bash scripts/gpu_suite.sh r04_closing || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_closing/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r04_closing/smoke.log; exit 1; }
tail -1 gpurun_out/r04_closing/smoke.log
