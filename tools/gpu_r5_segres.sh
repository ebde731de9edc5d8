# round-5: the fused segment start (k_seg_resume): the loop suites (incl. the wide split's), a C3 bench, a HIP API + kernel trace
set -o pipefail
tag=${1:-segres}
bash tools/gpu_r5_loop.sh $tag || exit 1
timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 20 --warmup 2 > gpurun_out/r5_bench_$tag.json 2> gpurun_out/r5_bench_$tag.err || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 > gpurun_out/prof_${tag}_bench.json 2> gpurun_out/prof_${tag}_bench.err || exit 3
