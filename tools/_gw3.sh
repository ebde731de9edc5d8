cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "floww or wide or 512 or n300 or 200" > gpurun_out/gw_tests.log 2>&1
rc=$?; tail -8 gpurun_out/gw_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --cfg 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/c4.json')); print(round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gt_tests.log; grep -E "FAIL|Error" gpurun_out/gt_tests.log | head -5; exit $rc
