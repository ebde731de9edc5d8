#!/bin/bash
# round 4: where the new k_round2 spends its iteration -- realtime stamps
# (BH_DIAG timeline) of this build and of 9148f1d, and each loop alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label lib env...
  local lab=$1 lib=$2; shift 2
  if [ "$lib" = "-" ]; then
    env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err
  else
    env BH_LIB_PATH=$PWD/$lib "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/c4_$lab.json 2> gpurun_out/c4_$lab.err
  fi
  local rc=$?
  echo "== $lab rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/c4_$lab.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/c4_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
}
run tl_new - BH_DIAG=1 BH_TIMELINE=gpurun_out/tl_new.bin && python tools/timeline.py gpurun_out/tl_new.bin
run tl_old ab_libs/9148f1d.so BH_DIAG=1 BH_TIMELINE=gpurun_out/tl_old.bin && python tools/timeline.py gpurun_out/tl_old.bin
run ser_new - BH_SEG_SERIAL=1
run ser_old ab_libs/9148f1d.so BH_SEG_SERIAL=1
run eager_new - BH_EAGER_ROWS=1
run tlser_new - BH_SEG_SERIAL=1 BH_DIAG=1 BH_TIMELINE=gpurun_out/tlser_new.bin && python tools/timeline.py gpurun_out/tlser_new.bin
run tlser_old ab_libs/9148f1d.so BH_SEG_SERIAL=1 BH_DIAG=1 BH_TIMELINE=gpurun_out/tlser_old.bin && python tools/timeline.py gpurun_out/tlser_old.bin
