#!/bin/bash
# round 4: localise the wide la_col loop's round mismatch; n <= 128 parity with
# the 8-lane hand-off and the persistent loop; C3 A/B (per-iteration launches,
# persistent loop, round-3 row sources)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "base:X=0" "p16:BH_ROUND_P8=0" "p8win:BH_ROUND_P8G=0" "single:BH_ROUND_ILP2=0" "fdt:BH_WIDE_ROWS=1" "seg1:BH_SEGMENTS=1"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env BH_WIDE_COLS=1 $envs TAG=$lab timeout -k 10 120 python tools/dbg_wide.py 200 30000 74 || exit $?
done
BH_WIDE_COLS=1 TAG=n512 timeout -k 10 120 python tools/dbg_wide.py 512 25000 113 || exit $?
BH_WIDE_COLS=1 TAG=n300p16 BH_ROUND_P8=0 timeout -k 10 120 python tools/dbg_wide.py 300 30000 112 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -v --timeout 300 --timeout-method thread -rf \
  -k "persistent or la_col or small_n or random_dag or wild or lazy_rows or split or segment_pipeline_parity" > gpurun_out/r4_tests11.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests11.log | tail -2; grep FAILED gpurun_out/r4_tests11.log | head
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for spec in "col:X=0" "pers:BH_ROUND_PERSIST=1" "rows:BH_ROUND_SRC=rows" "col2:X=0" "pers2:BH_ROUND_PERSIST=1" "persser:BH_ROUND_PERSIST=1 BH_SEG_SERIAL=1" "colser:BH_SEG_SERIAL=1"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-sample 0 > gpurun_out/c11_$lab.json 2> gpurun_out/c11_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c11_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c11_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
exit 0
