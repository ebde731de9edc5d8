#!/bin/bash
# round-4 closing run: every GPU test, smoke, the default bench line (C3, cpu baseline included), the other
# BASELINE configs, rocprofv3 kernel stats and PMC traffic / SQ passes of C3 and C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit $?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
timeout -k 10 600 python bench.py > gpurun_out/final_c3.json 2> gpurun_out/final_c3.err || { echo "bench c3 failed"; tail -5 gpurun_out/final_c3.err; exit 1; }
cat gpurun_out/final_c3.json
for c in 2 5 4; do
  timeout -k 10 300 python bench.py --cfg $c --cpu-sample 0 > gpurun_out/final_c$c.json 2> gpurun_out/final_c$c.err || { echo "bench c$c failed"; tail -5 gpurun_out/final_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/final_c$c.json')); print('c$c', round(d['value']/1e6,2), round(d['ms_per_step'],2), d['stages_ms'])"
done
bash tools/prof.sh r4f_c4 --cfg 4 --steps 2 --warmup 1 || exit $?
bash tools/prof.sh r4f_c3 --cfg 3 --steps 3 --warmup 1 || exit $?
bash tools/pmc.sh r4fc4 "." --cfg 4 || exit $?
bash tools/pmc.sh r4fc3 "." --cfg 3 || exit $?
exit 0
