# round-5: segment count / ratio around the default with the faster loop, interleaved on one box
set -o pipefail
for k in 1 2; do
for cfg in "12 1.32" "12 1.28" "12 1.24" "14 1.28" "16 1.24"; do
set -- $cfg
BH_SEGMENTS=$1 BH_SEG_RATIO=$2 timeout -k 10 200 python3 bench.py --cpu-sample 0 --steps 15 --warmup 2 > gpurun_out/r5_seg_$1_$2_$k.json 2> gpurun_out/r5_seg_$1_$2_$k.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5_seg_$1_$2_$k.json')); print('K $1 ratio $2 run $k', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms loop', round(d['roofline']['loop']['us_per_iteration'],3))"
done
done
