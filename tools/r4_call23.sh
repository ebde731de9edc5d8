#!/bin/bash
# round 4 closing run: every GPU test, smoke, the default bench line (C3 with
# its CPU baseline, as the driver runs it) and the other BASELINE configs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rf > gpurun_out/r4_tests23.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests23.log | tail -2; grep FAILED gpurun_out/r4_tests23.log | head -20
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('default', round(d['value']/1e6,2), round(d['ms_per_step'],2), d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
for c in 2 5 4; do
  timeout -k 10 300 python bench.py --cfg $c --cpu-sample 0 > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo "cfg$c failed"; tail -5 gpurun_out/bench_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_c$c.json')); print('cfg$c', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['us_per_iteration'],2), d['stages_ms'])"
done
exit $rc
