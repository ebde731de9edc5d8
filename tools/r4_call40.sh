#!/bin/bash
# round 4: same-box A/B of engine builds at C4 -- HEAD (new rows prefetched ahead of the fit check), the build
# before it (prev), both with -falign-loops=64 (cur_al, prev_al): is the search's slowdown code placement?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--cfg 4 --steps 3 --warmup 1" bash tools/ab_libs.sh 2 - tools/ablib/prev.so tools/ablib/cur_al.so tools/ablib/prev_al.so || exit $?
BENCH_ARGS="--cfg 3 --steps 10 --warmup 1" bash tools/ab_libs.sh 1 - tools/ablib/cur_al.so || exit $?
exit 0
