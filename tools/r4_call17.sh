#!/bin/bash
# round 4: where the segments' Lamport timestamps run (combined / own stream /
# after the columns) at C3 / C5 / C2, XCD barrier at C5; parity of the LT modes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -rf -k "random_dag or segment or lt_fallback or persistent or trap or c3_multisegment or c5_whole" > gpurun_out/r4_tests17.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests17.log | tail -2; grep FAILED gpurun_out/r4_tests17.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c17_$lab.json 2> gpurun_out/c17_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c17_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c17_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c3 3 20 X=0
run c3lt0 3 20 BH_LT_MODE=0
run c3lt1 3 20 BH_LT_MODE=1
run c3b 3 20 X=0
run c5 5 20 X=0
run c5lt0 5 20 BH_LT_MODE=0
run c5lt2 5 20 BH_LT_MODE=2
run c5xcd 5 20 BH_PBAR=xcd
run c2 2 20 X=0
run c2lt0 2 20 BH_LT_MODE=0
exit 0
