# round-5: host waits (spin on hipStreamQuery, pinned staging): loop suites, two C3 benches, a kernel + copy trace
set -o pipefail
tag=${1:-host}
bash tools/gpu_r5_loop.sh $tag || exit 1
for i in 1 2; do
timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 20 --warmup 2 > gpurun_out/r5_bench_${tag}_$i.json 2> gpurun_out/r5_bench_${tag}_$i.err || exit 2
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 > gpurun_out/prof_${tag}_bench.json 2> gpurun_out/prof_${tag}_bench.err || exit 4
