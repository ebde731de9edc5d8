# A/B of env knobs on the C3 bench: bash tools/_ab_env.sh "LABEL:VAR=val VAR2=val" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 150 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/ab_$lab.json 2> gpurun_out/ab_$lab.err || { echo "$lab failed"; tail -5 gpurun_out/ab_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$lab.json')); print('$lab', round(d['value']/1e6,1), round(d['ms_per_step'],2), round(d['roofline']['dominant_kernel']['avg_launch_ms']*1e3,2), d.get('stages_ms'))"
done
