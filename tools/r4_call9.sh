#!/bin/bash
# round 4: LT race fix + one-load window / 32-bit hand-off; parity, col vs rows A/B, SQ instruction counts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_schedule.py tests/test_gpu_reset.py -m gpu -v --timeout 300 --timeout-method thread -rf \
  -k "random_dag or la_col or lazy_rows or split or kat_dag or trap_wide or small_n or segment or reset or lt_fallback or silent or wild" > gpurun_out/r4_tests9.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests9.log | tail -3; grep FAILED gpurun_out/r4_tests9.log | head
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for spec in "col:X=0" "rows:BH_ROUND_SRC=rows" "col2:X=0" "rows2:BH_ROUND_SRC=rows" "colser:BH_SEG_SERIAL=1" "rowsser:BH_ROUND_SRC=rows BH_SEG_SERIAL=1"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-sample 0 > gpurun_out/c9_$lab.json 2> gpurun_out/c9_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c9_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c9_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
for spec in "col:X=0" "rows:BH_ROUND_SRC=rows"; do
  lab=${spec%%:*}; envs=${spec#*:}
  out=gpurun_out/sq9_$lab; mkdir -p $out
  env $envs BH_NO_GRAPH=1 BH_SEG_SERIAL=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
    --kernel-include-regex "k_round2" --output-format csv -d $out -o run -- python bench.py --steps 1 --warmup 0 --cpu-sample 0 --quiet > $out/bench.json 2> $out/bench.err
  rc=$?; echo "sq $lab rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/bench.err; exit $rc; }
done
exit 0
