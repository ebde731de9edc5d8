# round-5: the loop's test suites, then a kernel + copy trace of the C3 bench (tools/gaps.py reads it)
set -o pipefail
tag=${1:-prof}
bash tools/gpu_r5_loop.sh $tag || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/prof_${tag}_bench.json 2> gpurun_out/prof_${tag}_bench.err || exit 2
