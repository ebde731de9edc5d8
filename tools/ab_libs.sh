#!/bin/bash
# Same-box A/B of engine builds, interleaved so box drift hits all of them:
#   BENCH_ARGS="--cfg 3 --steps 20 --warmup 2" bash tools/ab_libs.sh ROUNDS lib1.so lib2.so ...
# ("-" = the in-tree build).  One JSON line per run under gpurun_out/ab_<i>_<k>.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
args=${BENCH_ARGS:---steps 20 --warmup 2}
rounds=$1; shift
for k in $(seq 1 "$rounds"); do
  i=0
  for lib in "$@"; do
    out=gpurun_out/ab_${i}_$k.json
    if [ "$lib" = "-" ]; then
      timeout -k 10 200 python bench.py $args --cpu-sample 0 > "$out" 2> "${out%.json}.err"
    else
      BH_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py $args --cpu-sample 0 > "$out" 2> "${out%.json}.err"
    fi
    rc=$?
    if [ $rc -ne 0 ]; then echo "$lib failed rc=$rc"; tail -5 "${out%.json}.err"; exit $rc; fi
    python -c "import json,sys; d=json.load(open('$out')); print('$lib', 'run $k', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', 'loop us/round', round(d['roofline']['loop']['us_per_iteration'],3))"
    i=$((i+1))
  done
done
exit 0
