# round-5 GPU step: bench first (fail fast), a diag timeline, then the loop's parity tests
set -o pipefail
tag=${1:-x}
timeout -k 10 240 python bench.py --steps 20 --warmup 2 > gpurun_out/r5_bench_$tag.json 2> gpurun_out/r5_bench_$tag.err || exit 1
BH_DIAG=1 BH_TIMELINE=gpurun_out/r5_tl_$tag.bin timeout -k 10 120 python bench.py --steps 1 --warmup 0 --cpu-sample 0 > /dev/null 2> gpurun_out/r5_tl_$tag.err || exit 2
[ "${2:-tests}" = "notests" ] && exit 0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_whole.py::test_c3_whole_dag tests/test_gpu_fullsize.py tests/test_gpu_schedule.py tests/test_gpu_fuzz.py > gpurun_out/r5_tests_$tag.log 2>&1 || exit 3
