# Unprofiled bench.py under several environment settings.  Usage: bash scripts/ab_env.sh TAG "K=V K2=V2" ...
set -o pipefail
TAG=$1; shift
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ab_${TAG}_$i.json 2>gpurun_out/ab_${TAG}_$i.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$i.json')); r=d['roofline']; print('$envs', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; apply', round(r['avg_launch_us'],1), 'us')"
done
