#!/bin/bash
# A/B of library builds in one GPU session: tools/ab.sh <bench args> -- lib1.so lib2.so ...
# (the in-tree build first, then each alternative via BH_LIB_PATH)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
args=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
shift || true
i=0
for lib in "" "$@"; do
  out=gpurun_out/ab_$i.log
  if [ -z "$lib" ]; then
    timeout -k 10 300 python bench.py --cpu-sample 0 "${args[@]}" > $out 2>&1
  else
    BH_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --cpu-sample 0 "${args[@]}" > $out 2>&1
  fi
  rc=$?
  echo "== ${lib:-in-tree} rc=$rc"; grep -o '"stages_ms[^}]*' $out
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
