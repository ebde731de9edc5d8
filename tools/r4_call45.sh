#!/bin/bash
# round 4: the transpose walk's stores addressed from a scalar row base (tools/ablib/sc.so) -- FD parity with that
# build, then same-box C4 A/B against HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BH_LIB_PATH=$PWD/tools/ablib/sc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -rf -k "transpose_fd_walk or coordinates_random or fdt_p8" > gpurun_out/r4_tests45.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests45.log | tail -1
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_ARGS="--cfg 4 --steps 3 --warmup 1" bash tools/ab_libs.sh 2 - tools/ablib/sc.so || exit $?
exit 0
