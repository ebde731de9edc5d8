# round-5 counters: PMC HBM bytes + SQ counters of one bench step at C3 and C4,
# and the kernel-trace stats of C3 (direct launches)
set -o pipefail
bash tools/pmc.sh c3 '.*' --cfg 3 || exit 1
bash tools/pmc.sh c4 '.*' --cfg 4 || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5c3 -o run -- python bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/prof_r5c3_bench.json 2> gpurun_out/prof_r5c3_bench.err || exit 3
timeout -k 10 300 python bench.py --cfg 4 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/r5_bench_c4.json 2> gpurun_out/r5_bench_c4.err || exit 4
