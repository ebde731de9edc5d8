#!/bin/bash
# round 4: barrier-phase stamps (BH_DIAG second block: end, arrived, staged, released, every workgroup) --
# C4 persistent wide loop with / without prestage, C3 k_round2p; quick wide parity first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -rf -k "wide_parity or persistent" > gpurun_out/r4_tests30.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests30.log | tail -2; grep -E "FAILED|Error" gpurun_out/r4_tests30.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
tl() {  # label cfg env...
  local lab=$1 cfg=$2; shift 2
  env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl30_$lab.bin "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c30_$lab.json 2> gpurun_out/c30_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c30_$lab.err; exit 1; }
  echo "== $lab"; python tools/timeline.py gpurun_out/tl30_$lab.bin
}
tl c4 4 X=0
tl c4nopre 4 BH_PRESTAGE=0
tl c3 3 X=0
exit 0
