#!/bin/bash
# round 4: parity of the cla / priority build, then k_round2 wave-priority A/B at C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_schedule.py -m gpu -v --timeout 300 --timeout-method thread -rf \
  -k "random_dag or la_col or lazy_rows or split_pipeline or kat_dag or trap_wide or small_n" > gpurun_out/r4_tests5.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/r4_tests5.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
for spec in "p0:BH_ROUND_PRIO=0" "p1:BH_ROUND_PRIO=1" "p3:BH_ROUND_PRIO=3" "p0b:BH_ROUND_PRIO=0" "p3b:BH_ROUND_PRIO=3"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-sample 0 > gpurun_out/c5_$lab.json 2> gpurun_out/c5_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c5_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
env BH_DIAG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5_diag.json 2> gpurun_out/c5_diag.err; grep "bh diag" gpurun_out/c5_diag.err | tail -4
