#!/bin/bash
# round 4: k_round_wide with its probe loop rolled (#pragma unroll 1: kernel 45.5 -> 37.5 KB) against HEAD, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--cfg 4 --steps 3 --warmup 1" bash tools/ab_libs.sh 2 - tools/ablib/roll.so || exit $?
exit 0
