# round-5: the other configs under the default pipeline vs the round-4 ratio (BH_SEG_RATIO=1.5), one box
set -o pipefail
out=gpurun_out/r5_cfgs.txt
: > $out
for cfg in 3 5 2 5 2 3; do
  for r in 1.38 1.5; do
    BH_SEG_RATIO=$r timeout -k 10 180 python bench.py --cfg $cfg --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/r5_cfg${cfg}_$r.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r5_cfg${cfg}_$r.json')); print('cfg$cfg ratio=$r', round(d['ms_per_step'],3), round(d['value']/1e6,1), d['pipeline'])" | tee -a $out
  done
done
