# the -m gpu suite in reverse order (state left in module-scoped fixtures)
set -u
mkdir -p gpurun_out/r04_reverse
PYTHONPATH=scripts timeout -k 10 900 python -u -m pytest tests -m gpu -p pytest_reverse -q --maxfail=10 --timeout 300 --timeout-method thread \
  > gpurun_out/r04_reverse/pytest_gpu_reverse.log 2>&1
rc=$?
tail -3 gpurun_out/r04_reverse/pytest_gpu_reverse.log
[ $rc -le 1 ] || exit $rc
