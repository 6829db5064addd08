set -u
timeout -k 10 300 python -u -m pytest tests/test_peak_detect.py tests/test_dist_gpu.py tests/test_website_fixture.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04_peak_tests3.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r04_peak_tests3.log; exit 1; }
tail -1 gpurun_out/r04_peak_tests3.log
rm -rf gpurun_out/r04_dyn_rt
bash scripts/gpu_r04_c16.sh > /dev/null || exit 1
python3 scripts/dyn_gap_summary.py gpurun_out/r04_dyn_rt/trace | head -3
bash scripts/gpu_r04_c11.sh | grep -E "k_tile|k_peak" || exit 1
grep '"metric"' gpurun_out/r04_dyn/trace.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l[l.index('{'):]); print('ms_per_step', d['ms_per_step'])"
