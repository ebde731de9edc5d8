cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t9.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t9.log; [ $rc -ne 0 ] && exit $rc
for c in 2 5; do for K in 1 4; do BH_SEGMENTS=$K timeout -k 10 300 python bench.py --cfg $c --steps 3 --cpu-sample 0 > gpurun_out/b9.json 2> gpurun_out/b9.err || exit 1; python -c "
import json; d=json.load(open('gpurun_out/b9.json')); print('cfg$c K=$K', round(d['value']/1e6,1), round(d['ms_per_step'],2), d['stages_ms'])"; done; done
