# GPU box: the host-ahead diagnostic (bench.py --host-ahead): GPU-side step time with every step
# enqueued before the GPU reaches it, for the 1-GPU line and rank 0 of 8 emulated.
# Usage: bash scripts/gpu_ahead.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
for sh in 0 1; do
  RG_OWNER_ITEM_SHARD=$sh timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 --host-ahead 30 > gpurun_out/ahead_emul_${TAG}_is$sh.json 2>gpurun_out/ahead_emul_${TAG}_is$sh.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/ahead_emul_${TAG}_is$sh.json'));print('emul is$sh ahead', round(d['gpu_ahead_us_per_step'],2), 'host', round(d['host_enqueue_us_per_step'],2))"
done
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --host-ahead 30 > gpurun_out/ahead_b_$TAG.json 2>gpurun_out/ahead_b_$TAG.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/ahead_b_$TAG.json'));print('1gpu ahead', round(d['gpu_ahead_us_per_step'],2), 'host', round(d['host_enqueue_us_per_step'],2))"
