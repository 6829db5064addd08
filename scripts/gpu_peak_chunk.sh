set -u -o pipefail
mkdir -p gpurun_out/pk_chunk
timeout -k 10 300 python -u -m pytest tests/test_peak_detect.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pk_chunk/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pk_chunk/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_peak_chunk.py 0 1 2 4 8 > gpurun_out/pk_chunk/ab.log 2>&1 || { tail -5 gpurun_out/pk_chunk/ab.log; exit 1; }
tail -1 gpurun_out/pk_chunk/ab.log
