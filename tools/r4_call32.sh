#!/bin/bash
# round 4: k_round_wide priorities (BH_WIDE_PRIO=1: hand-off / barrier / next window's staging at priority 2;
# 2: also the two workgroups of a CU alternate priority pass by pass) -- parity, C4 A/B, timelines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -rf -k "transpose_fd_walk or wide_parity" > gpurun_out/r4_tests32.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests32.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests32.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 1 --cpu-sample 0 > gpurun_out/c32_$lab.json 2> gpurun_out/c32_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c32_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c32_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c4 4 5 X=0
run c4p1 4 5 BH_WIDE_PRIO=1
run c4p2 4 5 BH_WIDE_PRIO=2
run c4b 4 5 X=0
run c4p1b 4 5 BH_WIDE_PRIO=1
for m in 1 2; do
env BH_WIDE_PRIO=$m BH_DIAG=1 BH_TIMELINE=gpurun_out/tl32_p$m.bin timeout -k 10 200 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c32_tl$m.json 2> gpurun_out/c32_tl$m.err || { echo "tl failed"; exit 1; }
echo "== prio $m"; python tools/timeline.py gpurun_out/tl32_p$m.bin
done
exit 0
