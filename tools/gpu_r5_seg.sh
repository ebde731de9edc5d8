# round-5 sweep: segment count x geometric ratio of the pipeline (C3, one box)
set -o pipefail
out=gpurun_out/r5_seg_sweep.txt
: > $out
IFS=, read -ra CFGS <<< "${SWEEP:-8 1.5,10 1.5,12 1.4,10 1.35,12 1.3,16 1.25,8 1.5}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  BH_SEGMENTS=$1 BH_SEG_RATIO=$2 timeout -k 10 180 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/r5_seg_$1_$2.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r5_seg_$1_$2.json')); print('K=$1 ratio=$2', round(d['ms_per_step'],2), round(d['value']/1e6,1), round(d['roofline']['loop']['us_per_iteration'],3), d['stages_ms'])" | tee -a $out
done
