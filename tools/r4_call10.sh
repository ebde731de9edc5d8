#!/bin/bash
# round 4: the wide loop over la_col (no FDT / row-major LA at C4); C4 A/B, then wide parity
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -rf -k "wide_parity" > gpurun_out/r4_tests10a.log 2>&1
rc=$?
echo "wide parity rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests10a.log | tail -2; grep FAILED gpurun_out/r4_tests10a.log | head
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for spec in "cols:X=0" "fdt:BH_WIDE_ROWS=1"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --cfg 4 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/c10_$lab.json 2> gpurun_out/c10_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c10_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c10_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_whole.py tests/test_gpu_shard.py tests/test_gpu_schedule.py tests/test_gpu_query.py -m gpu -v --timeout 600 --timeout-method thread -rf \
  -k "(wide and not wide_parity) or 512 or long_chains or trap or group or query or lazy or c4_whole" > gpurun_out/r4_tests10.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests10.log | tail -3; grep FAILED gpurun_out/r4_tests10.log | head
exit $rc
