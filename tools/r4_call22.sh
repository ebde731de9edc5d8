#!/bin/bash
# round 4: closing profiles -- host-ASan engine run over the host paths,
# incremental (gossip) calls at n = 128 / 512 with the persistent loops,
# rocprofv3 kernel stats and PMC traffic / SQ counters of C3 and C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 bash tools/sanitize_engine.sh -m gpu -q -x --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_reset.py tests/test_gpu_shard.py tests/test_gpu_frames.py tests/test_gpu_query.py \
  -k "not full_size and not large_properties and not wide_parity and not long_chains and not whole" > gpurun_out/r4_sanitize.log 2>&1
rc=$?
echo "sanitize rc=$rc"; tail -3 gpurun_out/r4_sanitize.log; ls gpurun_out | grep -E "^asan|^ubsan" | head
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for n in 128 512; do
  timeout -k 10 200 python tools/bench_gossip.py --n $n --events 1100000 --batch 1000 --prefill 1000000 > gpurun_out/gossip_n$n.json 2> gpurun_out/gossip_n$n.err || { echo "gossip $n failed"; tail -3 gpurun_out/gossip_n$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/gossip_n$n.json')); print('gossip n=$n', d['consensus_ms_median'], d['consensus_ms_max'], d['incremental_calls'])"
done
BH_ROUND_PERSIST=0 timeout -k 10 200 python tools/bench_gossip.py --n 128 --events 1100000 --batch 1000 --prefill 1000000 > gpurun_out/gossip_n128_it.json 2> gpurun_out/gossip_n128_it.err && python -c "import json; d=json.load(open('gpurun_out/gossip_n128_it.json')); print('gossip n=128 per-iteration', d['consensus_ms_median'], d['consensus_ms_max'])"
bash tools/prof.sh r4_c4 --cfg 4 --steps 2 --warmup 1 || exit $?
bash tools/pmc.sh r4c4 "." --cfg 4 || exit $?
bash tools/prof.sh r4_c3f --cfg 3 --steps 3 --warmup 1 || exit $?
bash tools/pmc.sh r4c3f "." --cfg 3 || exit $?
exit 0
