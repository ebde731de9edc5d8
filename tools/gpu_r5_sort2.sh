# round-5: the two-pass frame sort: the order / frame / whole-DAG suites, a C3 bench and its kernel stats
set -o pipefail
tag=${1:-sort2}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_whole.py tests/test_gpu_shard.py tests/test_gpu_reset.py -m gpu > gpurun_out/r5_tests_$tag.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 20 --warmup 2 > gpurun_out/r5_bench_$tag.json 2> gpurun_out/r5_bench_$tag.err || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/prof_${tag}_bench.json 2> gpurun_out/prof_${tag}_bench.err || exit 3
timeout -k 10 300 python3 bench.py --cfg 4 --cpu-sample 0 --steps 5 --warmup 1 > gpurun_out/r5_bench_${tag}_c4.json 2> gpurun_out/r5_bench_${tag}_c4.err || exit 4
