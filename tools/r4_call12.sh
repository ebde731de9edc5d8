#!/bin/bash
# round 4 (session 2): state of HEAD -- every GPU test, smoke, then C3 and C4 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rf > gpurun_out/r4_tests12.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4_tests12.log | tail -2; grep FAILED gpurun_out/r4_tests12.log | head -20
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for c in 3 4; do
  timeout -k 10 200 python bench.py --cfg $c --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/c12_$c.json 2> gpurun_out/c12_$c.err || { echo "cfg$c failed"; tail -5 gpurun_out/c12_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c12_$c.json')); print('cfg$c', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d['stages_ms'])"
done
exit $rc
