cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t10.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t10.log; grep -E "FAIL|Error" gpurun_out/t10.log | head -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --cpu-sample 0 > gpurun_out/b10.json 2> gpurun_out/b10.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/b10.json')); print(round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'])"
timeout -k 10 300 python tools/bench_gossip.py --n 128 --events 1100000 --prefill 1000000 --batch 1000 > gpurun_out/g10a.json 2> gpurun_out/g10a.err || exit 1; cat gpurun_out/g10a.json
timeout -k 10 300 python tools/bench_gossip.py --n 32 --events 1050000 --prefill 1000000 --batch 500 > gpurun_out/g10b.json 2> gpurun_out/g10b.err || exit 1; cat gpurun_out/g10b.json
