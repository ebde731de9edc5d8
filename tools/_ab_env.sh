# A/B of env knobs on a bench config: [BENCH_ARGS="--cfg 4 --steps 2"] bash tools/_ab_env.sh "LABEL:VAR=val VAR2=val" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
args=${BENCH_ARGS:---steps 5 --warmup 1}
for spec in "$@"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 150 python bench.py $args --cpu-sample 0 > gpurun_out/ab_$lab.json 2> gpurun_out/ab_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/ab_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$lab.json')); print('$lab', round(d['value']/1e6,1), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d.get('stages_ms'))"
done
