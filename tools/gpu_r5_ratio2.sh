# round-5: the segment ratio again with the faster loop (BH_SEG_RATIO), interleaved on one box
set -o pipefail
for k in 1 2; do
for r in 1.38 1.45 1.52; do
BH_SEG_RATIO=$r timeout -k 10 200 python3 bench.py --cpu-sample 0 --steps 15 --warmup 2 > gpurun_out/r5_ratio_${r}_$k.json 2> gpurun_out/r5_ratio_${r}_$k.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5_ratio_${r}_$k.json')); print('ratio $r run $k', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms loop', round(d['roofline']['loop']['us_per_iteration'],3))"
done
done
