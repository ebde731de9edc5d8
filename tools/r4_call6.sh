#!/bin/bash
# round 4: is the loop's slowdown beside the coordinates CU sharing?  (timing A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "base:X=0" "nolt:BH_EXP_NOLT=1" "cu128:BH_CU_SPLIT=128" "nolt_cu128:BH_EXP_NOLT=1 BH_CU_SPLIT=128" "serial:BH_SEG_SERIAL=1" "nolt_cu136:BH_EXP_NOLT=1 BH_CU_SPLIT=136" "base2:X=0"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-sample 0 > gpurun_out/c6_$lab.json 2> gpurun_out/c6_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c6_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c6_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
