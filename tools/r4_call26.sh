#!/bin/bash
# round 4: C3's coordinate pipeline gates the loop -- LT beside the columns
# (BH_LT_MODE=1/2) with the persistent loop's waves at a higher priority
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c26_$lab.json 2> gpurun_out/c26_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c26_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c26_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run base 3 20 X=0
run lt1p3 3 20 BH_LT_MODE=1 BH_ROUND_PRIO=3
run lt2p3 3 20 BH_LT_MODE=2 BH_ROUND_PRIO=3
run lt1p1 3 20 BH_LT_MODE=1 BH_ROUND_PRIO=1
run lt1 3 20 BH_LT_MODE=1
run p3 3 20 BH_ROUND_PRIO=3
run base2 3 20 X=0
exit 0
