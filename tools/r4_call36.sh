#!/bin/bash
# round 4: wide transpose tile height A/B (BH_XPOSE_TR=64: one workgroup per CU, 64 entries per column and tile)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 env BH_XPOSE_TR=64 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -rf -k "transpose_fd_walk or fdt_p8 or fdt_p16" > gpurun_out/r4_tests36.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests36.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests36.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 1 --cpu-sample 0 > gpurun_out/c36_$lab.json 2> gpurun_out/c36_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c36_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c36_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c4 4 5 X=0
run c4tr64 4 5 BH_XPOSE_TR=64
run c4tr16 4 5 BH_XPOSE_TR=16
run c4b 4 5 X=0
run c4tr64b 4 5 BH_XPOSE_TR=64
exit 0
