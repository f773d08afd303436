# GPU box: lazy-pass timing experiments (RG_LAZY_DBG bits, wrong results) -- dense-pass event time.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
for v in "RG_LAZY=0" "RG_LAZY_SPEC=1 RG_LAZY_DBG=1" "RG_LAZY_SPEC=1 RG_LAZY_DBG=3" "RG_LAZY_SPEC=1 RG_LAZY_DBG=13" "RG_LAZY_SPEC=1 RG_LAZY_DBG=15" "RG_LAZY_SPEC=0 RG_LAZY_DBG=3" "RG_LAZY_SPEC=1 RG_LAZY_DBG=12"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $v timeout -k 10 200 python3 bench.py --gpus 1 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/b_${TAG}_$tag.json 2>>gpurun_out/b_$TAG.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_$tag.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2))"
done
