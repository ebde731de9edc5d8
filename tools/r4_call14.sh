#!/bin/bash
# round 4: wide loop window/hand-off source A/B at C4 (rows / la_col / window
# rows + la_col hand-off), C3 persistent-loop A/B, rocprofv3 stats and PMC
# traffic of C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -rf -k "wide_parity and cols2" > gpurun_out/r4_tests14.log 2>&1
rc=$?
echo "cols2 parity rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests14.log | tail -2; grep FAILED gpurun_out/r4_tests14.log | head
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 1 --cpu-sample 0 > gpurun_out/c14_$lab.json 2> gpurun_out/c14_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c14_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c14_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
}
run c4rows 4 5 X=0
run c4cols2 4 5 BH_WIDE_COLS=2
run c4cols 4 5 BH_WIDE_COLS=1
run c4cols2b 4 5 BH_WIDE_COLS=2
run c3base 3 20 X=0
run c3pers 3 20 BH_ROUND_PERSIST=1
run c3base2 3 20 X=0
run c3pers2 3 20 BH_ROUND_PERSIST=1
run c3persser 3 10 BH_ROUND_PERSIST=1 BH_SEG_SERIAL=1
run c3baseser 3 10 BH_SEG_SERIAL=1
bash tools/prof.sh r4_c3 --cfg 3 --steps 3 --warmup 1 || exit $?
bash tools/pmc.sh r4c3 "." --cfg 3 || exit $?
exit 0
