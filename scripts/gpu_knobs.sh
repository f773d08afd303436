# GPU box: same-box sweep of MF bench env knobs, interleaved rounds.
# Usage: bash scripts/gpu_knobs.sh TAG "ENV_A" "ENV_B" ...   (each ENV is "K=V K2=V2", or "-" for none)
set -o pipefail
TAG=${1:-knobs}; shift
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for k in 1 2; do
  for cfg in "$@"; do
    e=$cfg; [ "$e" = "-" ] && e="RG_X=0"
    env $e timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/k_$TAG.json 2>/dev/null || exit $?
    echo "$cfg :" $(tail -1 gpurun_out/k_$TAG.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; ev', round(d['roofline']['avg_launch_us'],1), 'us')")
  done
done
