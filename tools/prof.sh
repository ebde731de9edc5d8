#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench configuration.
# usage: tools/prof.sh <tag> <bench args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export BH_NO_GRAPH=${BH_NO_GRAPH:-1}
tag=$1; shift
mkdir -p gpurun_out/prof_$tag
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python bench.py --cpu-sample 0 "$@" > gpurun_out/prof_$tag/bench.json 2> gpurun_out/prof_$tag/bench.err
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof_$tag -name "*stats*" | head
exit $rc
