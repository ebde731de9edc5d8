# round-5: C3 whole-DAG test, the kernel/copy trace of the C3 bench, and an A/B of the frame sort's share
set -o pipefail
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread "tests/test_gpu_whole.py::test_c3_whole_dag" -m gpu > gpurun_out/r5_tests_c3w.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_seg12 -o run -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/prof_seg12_bench.json 2> gpurun_out/prof_seg12_bench.err || exit 2
BENCH_ARGS="--steps 10 --warmup 2" bash tools/ab_libs.sh 2 ablibs/cur.so ablibs/nobitonic.so > gpurun_out/r5_ab_sort.txt 2>&1 || exit 3
for f in gpurun_out/ab_0_1.json gpurun_out/ab_1_1.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['stages_ms'])" >> gpurun_out/r5_ab_sort.txt; done
