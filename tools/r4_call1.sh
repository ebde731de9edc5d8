#!/bin/bash
# round 4, first GPU session: the new parity tests, then the same-box A/B of
# the round-3 builds (headline regression check)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_whole.py tests/test_gpu_parity.py tests/test_gpu_reset.py tests/test_gpu_shard.py -m gpu -v \
  --timeout 600 --timeout-method thread -rf -k "split or group or la_col or lazy_rows or small_n or random_dag or kat_dag or whole or long_chains or per_sync_trap_512 or watchdog or wide_parity or allocation_failure or segments" \
  > gpurun_out/r4_tests1.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -25 gpurun_out/r4_tests1.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
exit $rc
