# GPU box: lazy-pass timing experiments (RG_LAZY_DBG bits; wrong results) vs the product and eager.
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "RG_LAZY_DBG=0" "RG_LAZY_DBG=1" "RG_LAZY=0"; do
  env $v timeout -k 10 300 python3 bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_${TAG}_${v}.json 2>>gpurun_out/b_$TAG.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d.get('lazy_dense_pass',{}).get('user_rows_per_step'))"
done
