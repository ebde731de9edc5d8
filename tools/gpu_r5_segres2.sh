# round-5: loops launched with their own timing events, k_seg_resume; A/B of the host wait mode (HSA_ENABLE_INTERRUPT=0)
set -o pipefail
tag=${1:-segres2}
bash tools/gpu_r5_loop.sh $tag || exit 1
for i in 1 2; do
timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 20 --warmup 2 > gpurun_out/r5_bench_${tag}_def$i.json 2> gpurun_out/r5_bench_${tag}_def$i.err || exit 2
HSA_ENABLE_INTERRUPT=0 timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 20 --warmup 2 > gpurun_out/r5_bench_${tag}_poll$i.json 2> gpurun_out/r5_bench_${tag}_poll$i.err || exit 3
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 > gpurun_out/prof_${tag}_bench.json 2> gpurun_out/prof_${tag}_bench.err || exit 4
