#!/bin/bash
# round 4: split tests, the same-box A/B of round-3 builds vs this one, rocprofv3 stats of C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -v --timeout 300 --timeout-method thread -rf -k "split" \
  > gpurun_out/r4_tests3.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r4_tests3.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
BENCH_ARGS="--steps 20 --warmup 2" bash tools/ab_libs.sh 1 ab_libs/r3head.so ab_libs/1a1c1cd.so - ab_libs/9148f1d.so ab_libs/9e42a74.so ab_libs/r3head.so ab_libs/1a1c1cd.so - || exit $?
bash tools/prof.sh r4_c3 --cfg 3 --steps 3 --warmup 1
