#!/bin/bash
# round 4: the wide loop's byte window with a bank-conflict-free layout (piece
# u of lane part at u LPC + part, odd candidate groups rotated) -- wide parity,
# C3 whole DAG (8 segments again), C4 A/B + SQ counters of k_round_wide
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_whole.py tests/test_gpu_schedule.py -m gpu -x -v --timeout 400 --timeout-method thread -rf -k "wide or 512 or c3_whole or 300 or 160" > gpurun_out/r4_tests29.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests29.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests29.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 1 --cpu-sample 0 > gpurun_out/c29_$lab.json 2> gpurun_out/c29_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c29_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c29_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c4 4 5 X=0
run c4b 4 5 X=0
out=gpurun_out/sq29; mkdir -p $out
BH_NO_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  --kernel-include-regex "k_round_wide" --output-format csv -d $out -o run -- python bench.py --cfg 4 --steps 1 --warmup 0 --cpu-sample 0 --quiet > $out/bench.json 2> $out/bench.err
echo "sq rc=$?"
exit 0
