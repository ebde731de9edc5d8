#!/bin/bash
# rocprofv3 PMC passes over one bench step (direct launches), one counter
# group per run as MI355X_MICROARCH.md's rocprofv3 section prescribes.
# usage: tools/pmc.sh <tag> <kernel-regex> <bench args...>
# (PMC_CMD="python tools/bench_reset.py --steps 1": another program instead of
# one bench.py step; the bench args are then appended to it)
# Writes gpurun_out/pmc_<tag>/p<i>/... ; stops at the first failing pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export BH_NO_GRAPH=1
tag=$1; kre=$2; shift 2
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
)
i=0
for p in "${passes[@]}"; do
  out=gpurun_out/pmc_$tag/p$i
  mkdir -p $out
  echo "pass $i: $p"
  timeout -s KILL 240 rocprofv3 --pmc $p --kernel-include-regex "$kre" --output-format csv -d $out -o run -- \
    ${PMC_CMD:-python bench.py --steps 1 --warmup 0 --cpu-sample 0 --quiet} "$@" > $out/bench.json 2> $out/bench.err
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $out/bench.err; exit $rc; }
  i=$((i+1))
done
exit 0
