#!/bin/bash
# round 4: same-box A/B of the round-3 builds against this one (headline regression check)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS="--steps 20 --warmup 2" bash tools/ab_libs.sh 1 ab_libs/r3head.so ab_libs/1a1c1cd.so - ab_libs/9148f1d.so ab_libs/9e42a74.so ab_libs/r3head.so ab_libs/1a1c1cd.so -
