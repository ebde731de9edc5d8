#!/bin/bash
# round 4: LT after each segment's columns (128 column workgroups beside the loop); parity, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_schedule.py tests/test_gpu_reset.py -m gpu -v --timeout 300 --timeout-method thread -rf \
  -k "random_dag or la_col or lazy_rows or split or kat_dag or trap_wide or small_n or segment or reset or lt_fallback or silent" > gpurun_out/r4_tests7.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/r4_tests7.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for spec in "col:X=0" "rows:BH_ROUND_SRC=rows" "col2:X=0" "rows2:BH_ROUND_SRC=rows" "colser:BH_SEG_SERIAL=1" "rowsser:BH_ROUND_SRC=rows BH_SEG_SERIAL=1"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-sample 0 > gpurun_out/c7_$lab.json 2> gpurun_out/c7_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c7_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c7_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
