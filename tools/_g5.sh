cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 170 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 60 --timeout-method thread -k "segment" > gpurun_out/t5.log 2>&1
rc=$?; echo "seg tests rc=$rc"; tail -15 gpurun_out/t5.log
[ $rc -ne 0 ] && exit $rc
for K in 1 2 4 8; do BH_SEGMENTS=$K timeout -k 10 300 python bench.py --steps 3 --cpu-sample 0 > gpurun_out/b5_$K.json 2> gpurun_out/b5_$K.err || exit 1; python -c "
import json; d=json.load(open('gpurun_out/b5_$K.json')); print($K, round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'])"; done
