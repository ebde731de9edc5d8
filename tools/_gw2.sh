cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_query.py -x -q --timeout 120 --timeout-method thread -k "floww or wide or 512 or random_pairs or full_size" > gpurun_out/gw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gw_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --cfg 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/c4.json')); print(round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'], d['roofline_coordinates']['avg_launch_ms'])"
BH_DIAG=1 timeout -k 10 300 python bench.py --cfg 4 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4d.json 2> gpurun_out/c4d.err; grep "k_flow wave0" gpurun_out/c4d.err | tail -1
