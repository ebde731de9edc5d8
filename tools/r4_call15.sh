#!/bin/bash
# round 4: persistent loop as the default -- every GPU test, bench lines of
# C3 / C2 / C5 / C4 (C2 / C5 with per-iteration launches beside), rocprofv3
# stats and PMC traffic of C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rf > gpurun_out/r4_tests15.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests15.log | tail -2; grep FAILED gpurun_out/r4_tests15.log | head -30
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c15_$lab.json 2> gpurun_out/c15_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c15_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c15_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
}
run c3 3 20 X=0
run c2 2 20 X=0
run c2it 2 20 BH_ROUND_PERSIST=0
run c5 5 20 X=0
run c5it 5 20 BH_ROUND_PERSIST=0
run c4 4 5 X=0
bash tools/prof.sh r4_c3p --cfg 3 --steps 3 --warmup 1 || exit $?
bash tools/pmc.sh r4c3p "." --cfg 3 || exit $?
exit $rc
