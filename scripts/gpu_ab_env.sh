# GPU box: same-box A/B of bench.py under environment settings.  Usage: bash scripts/gpu_ab_env.sh TAG "ENV1" "ENV2" ... [-- bench args]
set -o pipefail
TAG=$1; shift
ENVS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done; [ "$1" == "--" ] && shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for i in "${!ENVS[@]}"; do
    env ${ENVS[$i]} timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab_${TAG}_${i}_$rep.json 2>gpurun_out/ab_${TAG}_${i}_$rep.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_${i}_$rep.json'));print('${ENVS[$i]}', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2))"
  done
done
