#!/bin/bash
# round 4: XCD-hierarchical grid barrier in the persistent loop (parity, C3
# A/B), and where a C4 k_round_wide round spends its time (realtime stamps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -rf -k "persistent or small_n or la_col or random_dag" > gpurun_out/r4_tests16.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests16.log | tail -2; grep FAILED gpurun_out/r4_tests16.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c16_$lab.json 2> gpurun_out/c16_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c16_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c16_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c3flat 3 20 X=0
run c3xcd 3 20 BH_PBAR=xcd
run c3flat2 3 20 X=0
run c3xcd2 3 20 BH_PBAR=xcd
run c3xcdser 3 10 BH_PBAR=xcd BH_SEG_SERIAL=1
run c3flatser 3 10 BH_SEG_SERIAL=1
run c2xcd 2 20 BH_PBAR=xcd
run c2flat 2 20 X=0
run c5 5 20 X=0
run c5it 5 20 BH_ROUND_PERSIST=0
env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl_c4.bin timeout -k 10 200 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c16_tl4.json 2> gpurun_out/c16_tl4.err || { echo "tl4 failed"; tail -5 gpurun_out/c16_tl4.err; exit 1; }
python tools/timeline.py gpurun_out/tl_c4.bin
exit 0
