#!/bin/bash
# round 4: localise the wide la_col loop's round mismatch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "base:X=0" "p16:BH_ROUND_P8=0" "p8win:BH_ROUND_P8G=0" "single:BH_ROUND_ILP2=0" "fdt:BH_WIDE_ROWS=1" "seg1:BH_SEGMENTS=1"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs TAG=$lab timeout -k 10 120 python tools/dbg_wide.py 200 30000 74 || exit $?
done
TAG=n512 timeout -k 10 120 python tools/dbg_wide.py 512 25000 113 || exit $?
TAG=n300p16 BH_ROUND_P8=0 timeout -k 10 120 python tools/dbg_wide.py 300 30000 112 || exit $?
