set -u
mkdir -p gpurun_out/r04_c2
timeout -k 10 120 ./scripts/gathermask > gpurun_out/r04_c2/gathermask.log 2>&1 || { echo gathermask failed; tail gpurun_out/r04_c2/gathermask.log; exit 1; }
cat gpurun_out/r04_c2/gathermask.log
timeout -k 10 300 python -u scripts/bisect_outputs.py c475d4e be3a3bb b35c620 c9a26f5 HEAD > gpurun_out/r04_c2/bisect.log 2>&1 || { echo bisect failed; tail -20 gpurun_out/r04_c2/bisect.log; exit 1; }
cat gpurun_out/r04_c2/bisect.log
bash scripts/prof_fetch_split.sh r04_c2/fetch_split > gpurun_out/r04_c2/fetch_split.log 2>&1 || { echo fetch split failed; tail -30 gpurun_out/r04_c2/fetch_split.log; exit 1; }
tail -5 gpurun_out/r04_c2/fetch_split.log
