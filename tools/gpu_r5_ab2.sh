# round-5: same-box A/B of two builds with their stage times (order, fame)
set -o pipefail
BENCH_ARGS="--steps 10 --warmup 2" bash tools/ab_libs.sh ${ROUNDS:-2} "$@" > gpurun_out/r5_ab2.txt 2>&1 || exit 1
for f in gpurun_out/ab_*_1.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],3), d['stages_ms'])" >> gpurun_out/r5_ab2.txt; done
