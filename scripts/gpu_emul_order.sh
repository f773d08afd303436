# GPU box: rank 0 of 8 emulated with the owner user update started after the backward / the item
# pull / the item exchange (RG_OWNER_USER_AFTER 0 / 1 / 2), twice each, wall and GPU-side time.
# Usage: bash scripts/gpu_emul_order.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
for rep in 1 2; do for a in 0 1 2; do
  RG_OWNER_USER_AFTER=$a timeout -k 10 300 python3 bench.py --gpus 1 --steps 60 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 > gpurun_out/emul_order_${TAG}_${a}_$rep.json 2>gpurun_out/emul_order_${TAG}_${a}_$rep.err || exit $?
  RG_OWNER_USER_AFTER=$a timeout -k 10 300 python3 bench.py --gpus 1 --steps 60 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 --host-ahead 30 > gpurun_out/emul_order_ahead_${TAG}_${a}_$rep.json 2>gpurun_out/emul_order_ahead_${TAG}_${a}_$rep.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/emul_order_${TAG}_${a}_$rep.json'));h=json.load(open('gpurun_out/emul_order_ahead_${TAG}_${a}_$rep.json'));print('after $a rep $rep', round(d['ms_per_step']*1e3,2), 'us/step; user update', round(d['user_update_us'],2), '| ahead', round(h['gpu_ahead_us_per_step'],2))"
done; done
