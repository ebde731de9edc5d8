#!/bin/bash
# round-3 closing run: GPU tests, smoke, bench lines of every BASELINE config
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_check.sh tests smoke || exit $?
for c in 3 2 5 4; do
  timeout -k 10 300 python bench.py --cfg $c > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err
  rc=$?; echo "bench cfg$c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
