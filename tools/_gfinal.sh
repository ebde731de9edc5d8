# full GPU suite, C3 bench (default args), C3 kernel trace, C4 + C2 + C5 bench lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f_tests.log; grep -E "FAIL|Error" gpurun_out/f_tests.log | head -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/f_bench_c3.json 2> gpurun_out/f_bench_c3.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/f_bench_c3.json')); print('C3', round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'], d['cpu_baseline'])"
for c in 2 5 4; do
  timeout -k 10 300 python bench.py --cfg $c --steps 3 --cpu-sample 0 > gpurun_out/f_bench_c$c.json 2> gpurun_out/f_bench_c$c.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/f_bench_c$c.json')); print('C$c', round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'])"
done
