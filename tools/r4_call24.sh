#!/bin/bash
# round 4: fame inputs / round table stored after the barrier arrival in both
# persistent loops -- parity (persistent, Reset, wide, shards), C3 / C4 A/B
# lines and the k_round2p round timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reset.py tests/test_gpu_shard.py tests/test_gpu_schedule.py -m gpu -v --timeout 300 --timeout-method thread -rf \
  -k "persistent or wide_parity or small_n or la_col or random_dag or reset or split or trap or kat" > gpurun_out/r4_tests24.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests24.log | tail -2; grep FAILED gpurun_out/r4_tests24.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c24_$lab.json 2> gpurun_out/c24_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c24_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c24_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c3 3 20 X=0
run c4 4 5 X=0
run c3b 3 20 X=0
run c5 5 20 X=0
env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl_c3p.bin BH_SEG_SERIAL=1 timeout -k 10 200 python bench.py --cfg 3 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c24_tl3.json 2> gpurun_out/c24_tl3.err || { echo "tl3 failed"; tail -5 gpurun_out/c24_tl3.err; exit 1; }
python tools/timeline.py gpurun_out/tl_c3p.bin
env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl_c3q.bin timeout -k 10 200 python bench.py --cfg 3 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c24_tl3q.json 2> gpurun_out/c24_tl3q.err || { echo "tl3q failed"; tail -5 gpurun_out/c24_tl3q.err; exit 1; }
python tools/timeline.py gpurun_out/tl_c3q.bin
exit 0
