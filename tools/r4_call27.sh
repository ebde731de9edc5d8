#!/bin/bash
# round 4: (1) the wide persistent loop with its hand-off counted in la_col and
# no FDT (BH_WIDE_COLS=2): parity, C4 A/B; (2) C3's segment schedule -- per-
# segment timings and the segment count / first-segment sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -rf -k "wide_parity and (cols or iter or p8)" > gpurun_out/r4_tests27.log 2>&1
rc=$?
echo "wide parity rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests27.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests27.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c27_$lab.json 2> gpurun_out/c27_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c27_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c27_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c4 4 5 X=0
run c4cols2 4 5 BH_WIDE_COLS=2
env BH_SEG_DEBUG=1 timeout -k 10 200 python bench.py --cfg 3 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c27_segdbg.json 2> gpurun_out/c27_segdbg.err; grep "^\[seg" gpurun_out/c27_segdbg.err | tail -9
run c3 3 20 X=0
run c3k12 3 20 BH_SEGMENTS=12
run c3k16 3 20 BH_SEGMENTS=16
run c3k6 3 20 BH_SEGMENTS=6
run c3f16 3 20 BH_SEG_FIRST=16
run c3f60 3 20 BH_SEG_FIRST=60
exit 0
