#!/bin/bash
# round 4: the spread of k_round_wide's per-candidate answers T_q (BH_DIAG T_q block, tools/tq_stats.py) at C4,
# and the C4 line of this build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl38.bin timeout -k 10 200 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c38_tl.json 2> gpurun_out/c38_tl.err || { echo "tl failed"; tail -3 gpurun_out/c38_tl.err; exit 1; }
python tools/tq_stats.py gpurun_out/tl38.bin
python tools/timeline.py gpurun_out/tl38.bin
timeout -k 10 200 python bench.py --cfg 4 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/c38_c4.json 2> gpurun_out/c38_c4.err || { echo "c4 failed"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c38_c4.json')); print('c4', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
exit 0
