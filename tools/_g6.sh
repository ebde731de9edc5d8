cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 170 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 60 --timeout-method thread -k "segment or full_size or random_dag" > gpurun_out/t6.log 2>&1
rc=$?; echo "seg tests rc=$rc"; tail -3 gpurun_out/t6.log
[ $rc -ne 0 ] && exit $rc
for cfg in "1 256" "4 256" "4 1000000" "8 256" "8 1000000" "12 512"; do set -- $cfg
BH_SEGMENTS=$1 BH_XPOSE_WG=$2 timeout -k 10 300 python bench.py --steps 3 --cpu-sample 0 > gpurun_out/b6.json 2> gpurun_out/b6.err || exit 1; python -c "
import json; d=json.load(open('gpurun_out/b6.json')); print('K=$1 wg=$2', round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'])"; done
