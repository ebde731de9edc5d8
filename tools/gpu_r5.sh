set -o pipefail
timeout -k 10 240 python bench.py --steps 20 --warmup 2 > gpurun_out/r5_bench_async.json 2> gpurun_out/r5_bench_async.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_r5async -o run -- python bench.py --cpu-sample 0 --steps 2 --warmup 1 > gpurun_out/prof_r5async_bench.json 2> gpurun_out/prof_r5async_bench.err || exit 2
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_whole.py::test_c3_whole_dag tests/test_gpu_fullsize.py tests/test_gpu_reset.py > gpurun_out/r5_tests_async.log 2>&1 || exit 3
