#!/bin/bash
# round 4: grid barrier with per-workgroup release words (the completing arriver releases everyone) -- wide parity (persistent default, per-round
# launches, barrier fallback), n = 512 / long chains / C4 whole DAG, then C4 A/B
# and the persistent loop's round timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -rf -k "wide_parity or persistent or small_n or la_col" > gpurun_out/r4_tests20a.log 2>&1
rc=$?
echo "wide parity rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests20a.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests20a.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_whole.py tests/test_gpu_shard.py tests/test_gpu_schedule.py tests/test_gpu_fullsize.py tests/test_gpu_reset.py -m gpu -v --timeout 500 --timeout-method thread -rf \
  -k "(wide and not wide_parity) or 512 or long_chains or c4 or 300 or 160 or floww" > gpurun_out/r4_tests20.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests20.log | tail -2; grep FAILED gpurun_out/r4_tests20.log | head
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 1 --cpu-sample 0 > gpurun_out/c20_$lab.json 2> gpurun_out/c20_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c20_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c20_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c4pers 4 5 X=0
run c3 3 20 X=0
run c5 5 20 X=0
run c2 2 20 X=0
run c2xcd 2 20 BH_PBAR=xcd
run c4pers2 4 5 X=0
run c3b 3 20 X=0
env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl_c4r.bin timeout -k 10 200 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c20_tl4.json 2> gpurun_out/c20_tl4.err || { echo "tl4 failed"; tail -5 gpurun_out/c20_tl4.err; exit 1; }
python tools/timeline.py gpurun_out/tl_c4r.bin
exit $rc
