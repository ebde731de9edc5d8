#!/bin/bash
# round 4: HEAD's build (== the same-box A/B's "prev") -- every GPU test, smoke, the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit $?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
timeout -k 10 600 python bench.py > gpurun_out/head_c3.json 2> gpurun_out/head_c3.err || { echo "bench failed"; tail -5 gpurun_out/head_c3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/head_c3.json')); print('c3', round(d['value']/1e6,2), round(d['ms_per_step'],2), d['stages_ms'])"
exit 0
