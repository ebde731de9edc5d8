#!/bin/bash
# round 4: instruction-cache counters of k_round_wide at C4 -- HEAD's build against the prefetch build whose search
# ran 4 us slower (tools/ablib/pf.so): is it instruction fetch?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp BH_NO_GRAPH=1
C="SQ_WAVES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_INSTS_VALU"
for v in head pf; do
  out=gpurun_out/ic_$v; mkdir -p $out
  if [ $v = head ]; then lib=""; else lib=$PWD/tools/ablib/pf.so; fi
  BH_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_round_wide" --output-format csv -d $out -o run -- \
    python bench.py --cfg 4 --steps 1 --warmup 0 --cpu-sample 0 --quiet > $out/bench.json 2> $out/bench.err
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/bench.err; exit $rc; }
done
exit 0
