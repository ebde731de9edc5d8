# round-5 A/B: k_round2p's packed-f32 search against the int32 one (same box), a diag timeline, then the loop's test suites
set -o pipefail
tag=${1:-f32}
for v in 1 0 1 0; do
  BH_ROUND_F32=$v timeout -k 10 180 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/r5_ab_${tag}_$v.json 2>> gpurun_out/r5_ab_${tag}.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r5_ab_${tag}_$v.json')); print('F32=$v', round(d['ms_per_step'],2), round(d['value']/1e6,1), round(d['roofline']['loop']['us_per_iteration'],3))" | tee -a gpurun_out/r5_ab_${tag}.txt
done
BH_DIAG=1 BH_TIMELINE=gpurun_out/r5_tl_$tag.bin timeout -k 10 120 python bench.py --steps 1 --warmup 0 --cpu-sample 0 > /dev/null 2> gpurun_out/r5_tl_$tag.err || exit 2
bash tools/gpu_r5_loop.sh $tag || exit 3
