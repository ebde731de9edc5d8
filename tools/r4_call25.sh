#!/bin/bash
# round 4: release words for the flat barrier too (the arrival completing the
# counter releases everyone) -- persistent parity, C3 flat / xcd A/B, C2, C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reset.py tests/test_gpu_shard.py -m gpu -v --timeout 300 --timeout-method thread -rf \
  -k "persistent or wide_parity or small_n or la_col or random_dag or reset or split" > gpurun_out/r4_tests25.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests25.log | tail -2; grep FAILED gpurun_out/r4_tests25.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # label cfg steps env...
  local lab=$1 cfg=$2 steps=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --cfg $cfg --steps $steps --warmup 2 --cpu-sample 0 > gpurun_out/c25_$lab.json 2> gpurun_out/c25_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/c25_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c25_$lab.json')); print('$lab', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
}
run c3xcd 3 20 X=0
run c3flat 3 20 BH_PBAR=flat
run c3xcd2 3 20 X=0
run c3flat2 3 20 BH_PBAR=flat
run c2flat 2 20 X=0
run c2xcd 2 20 BH_PBAR=xcd
run c5xcd 5 20 X=0
run c5flat 5 20 BH_PBAR=flat
run c4 4 5 X=0
run c4flat 4 5 BH_PBAR=flat
exit 0
