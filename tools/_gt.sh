# GPU check: full -m gpu suite, then a C3 bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gt_tests.log; grep -E "FAIL|Error" gpurun_out/gt_tests.log | head -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --cpu-sample 0 > gpurun_out/gt_bench.json 2> gpurun_out/gt_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/gt_bench.json')); print(round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'])"
