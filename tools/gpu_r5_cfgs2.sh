# round-5: C2 / C5 / C4 bench lines of the current build
set -o pipefail
for c in 2 5 4; do
timeout -k 10 300 python3 bench.py --cfg $c --cpu-sample 0 --steps 10 --warmup 2 > gpurun_out/r5_bench_cfg$c.json 2> gpurun_out/r5_bench_cfg$c.err || exit $c
python3 -c "import json; d=json.load(open('gpurun_out/r5_bench_cfg$c.json')); print('cfg $c', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms loop', round(d['roofline']['loop']['us_per_iteration'],3))"
done
