#!/bin/bash
# round 4: k_round_wide loads its next window's new rows ahead of the fit check (BH_STAGE_PF=0: after it)
# -- wide parity (incl. C4-size whole DAG), C4 A/B, timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_whole.py tests/test_gpu_schedule.py -m gpu -x -v --timeout 300 --timeout-method thread -rf -k "wide or 512 or c4 or 300 or 160" > gpurun_out/r4_tests39.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests39.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests39.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 1 --cpu-sample 0 > gpurun_out/c39_$lab.json 2> gpurun_out/c39_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c39_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c39_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c4 4 5 X=0
run c4nopf 4 5 BH_STAGE_PF=0
run c4b 4 5 X=0
run c4nopfb 4 5 BH_STAGE_PF=0
env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl39.bin timeout -k 10 200 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c39_tl.json 2> gpurun_out/c39_tl.err || { echo "tl failed"; exit 1; }
python tools/timeline.py gpurun_out/tl39.bin
exit 0
