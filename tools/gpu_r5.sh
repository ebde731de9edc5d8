# round-5 GPU step: bench first (fail fast), then the loop's parity tests
set -o pipefail
tag=${1:-x}
timeout -k 10 240 python bench.py --steps 20 --warmup 2 > gpurun_out/r5_bench_$tag.json 2> gpurun_out/r5_bench_$tag.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_whole.py::test_c3_whole_dag tests/test_gpu_fullsize.py tests/test_gpu_schedule.py tests/test_gpu_fuzz.py > gpurun_out/r5_tests_$tag.log 2>&1 || exit 3
