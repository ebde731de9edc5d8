# round-5 full check: the whole GPU suite, then the C3 bench and its rocprofv3 kernel stats
set -o pipefail
tag=${1:-full}
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread tests/ -m gpu > gpurun_out/r5_tests_$tag.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 20 --warmup 2 > gpurun_out/r5_bench_$tag.json 2> gpurun_out/r5_bench_$tag.err || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5_$tag -o run -- python bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/prof_r5_${tag}_bench.json 2> gpurun_out/prof_r5_${tag}_bench.err || exit 3
