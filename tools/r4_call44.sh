#!/bin/bash
# round 4, HEAD: host-ASan engine run over the host paths, and the per-call cost of the live node's schedule at
# n = 128 / 512 (1000-event calls on a resident 1M-event DAG)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/sanitize_engine.sh -m gpu -q -x --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_reset.py tests/test_gpu_shard.py tests/test_gpu_frames.py tests/test_gpu_query.py \
  -k "not full_size and not large_properties and not wide_parity and not long_chains and not whole" > gpurun_out/r4_sanitize_head.log 2>&1
rc=$?
echo "sanitize rc=$rc"; tail -3 gpurun_out/r4_sanitize_head.log; ls gpurun_out | grep -E "^asan|^ubsan" | head
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for n in 128 512; do
  timeout -k 10 200 python tools/bench_gossip.py --n $n --events 1100000 --batch 1000 --prefill 1000000 > gpurun_out/gossip_head_n$n.json 2> gpurun_out/gossip_head_n$n.err || { echo "gossip $n failed"; tail -3 gpurun_out/gossip_head_n$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/gossip_head_n$n.json')); print('gossip n=$n', d['consensus_ms_median'], d['consensus_ms_max'], d['incremental_calls'])"
done
exit 0
