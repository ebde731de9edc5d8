#!/bin/bash
# round 4 (session 2): Reset hashgraphs after the fame fix (cla rows only for
# rounds >= r0), then every other GPU test, then the C4 wide-loop A/B
# (256 / 512 threads, FDT rows / la_col)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reset.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 300 --timeout-method thread -rf -k "reset" > gpurun_out/r4_tests13a.log 2>&1
rc=$?
echo "reset tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests13a.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests13a.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rf -k "not reset" > gpurun_out/r4_tests13.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests13.log | tail -2; grep FAILED gpurun_out/r4_tests13.log | head -30
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for spec in "base:X=0" "nt512:BH_WIDE_NT=512" "cols:BH_WIDE_COLS=1" "colsnt512:BH_WIDE_COLS=1 BH_WIDE_NT=512"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python bench.py --cfg 4 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/c13_$lab.json 2> gpurun_out/c13_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c13_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c13_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
exit $rc
