set -u
mkdir -p gpurun_out/r04_c1
export H2S_PARITY_REPORT=$PWD/gpurun_out/r04_c1/parity.jsonl
timeout -k 10 600 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_preview.py tests/test_website_fixture.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_c1/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r04_c1/pytest.log; [ $rc -eq 0 ] || exit $rc
BENCH=1 TMS="hable bt.2390" bash scripts/gpu_ab.sh r04_c1 scripts/variants/libh2s_head.so scripts/variants/libh2s_head.so
