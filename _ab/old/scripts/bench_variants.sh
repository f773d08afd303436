# bench.py variants for launch-overhead diagnosis.  Usage: bash scripts/bench_variants.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
for v in "--events-every 1" "--events-every 8" "--events-every 1000000" "--no-prefetch"; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline $v > gpurun_out/bv_$TAG.json 2>gpurun_out/bv_$TAG.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/bv_$TAG.json')); r=d.get('roofline',{}); print('$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step host', round(d['host_enqueue_us_per_step'],1), 'apply', round(r.get('avg_launch_us',0),1))"
done
