#!/bin/bash
# round 4: k_flow_transpose's FD walk as a scatter (one lane per row and column; BH_XPOSE_WALK=0: the binary search),
# k_round_wide's P8 window loaded with its fit check (one round trip) -- FD walk / wide parity, C4 A/B + timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -rf -k "transpose_fd_walk or wide_parity or coordinates_random or persistent" > gpurun_out/r4_tests31.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests31.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests31.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 1 --cpu-sample 0 > gpurun_out/c31_$lab.json 2> gpurun_out/c31_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c31_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c31_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c4 4 5 X=0
run c4bs 4 5 BH_XPOSE_WALK=0
run c4b 4 5 X=0
env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl31_c4.bin timeout -k 10 200 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c31_tl.json 2> gpurun_out/c31_tl.err || { echo "tl failed"; exit 1; }
python tools/timeline.py gpurun_out/tl31_c4.bin
exit 0
