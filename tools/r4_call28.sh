#!/bin/bash
# round 4: each segment's LT after the next segment's columns, 16 segments at
# C3 -- segment / LT parity, C3 whole DAG, C3 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_fullsize.py tests/test_gpu_whole.py tests/test_gpu_shard.py -m gpu -v --timeout 400 --timeout-method thread -rf \
  -k "c3_whole or c3_multi or segment_pipeline" > gpurun_out/r4_tests28.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests28.log | tail -2; grep FAILED gpurun_out/r4_tests28.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c28_$lab.json 2> gpurun_out/c28_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c28_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c28_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c3 3 20 X=0
run c3k8 3 20 BH_SEGMENTS=8
run c3k24 3 20 BH_SEGMENTS=24
run c3b 3 20 X=0
run c5 5 20 X=0
run c2 2 20 X=0
exit 0
