cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "4 0" "4 1" "8 0"; do set -- $v
echo "=== K=$1 serial=$2"
BH_SEG_DEBUG=1 BH_SEG_SERIAL=$2 BH_SEGMENTS=$1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b7.json 2> gpurun_out/b7.err || exit 1
grep "seg " gpurun_out/b7.err | tail -$1; python -c "
import json; d=json.load(open('gpurun_out/b7.json')); print(round(d['ms_per_step'],2), d['stages_ms'])"; done
