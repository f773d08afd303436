# GPU box: rank 0 of 8 emulated, wall time and GPU-side time (--host-ahead), item update all-reduced
# (RG_OWNER_ITEM_SHARD=0), then with the HIP API trace for where the host time goes.
# Usage: bash scripts/gpu_emul_ahead.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 > gpurun_out/emul_$TAG.json 2>gpurun_out/emul_$TAG.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 --host-ahead 30 > gpurun_out/emul_ahead_$TAG.json 2>gpurun_out/emul_ahead_$TAG.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/emul_$TAG.json'));a=json.load(open('gpurun_out/emul_ahead_$TAG.json'));print('emul', round(d['ms_per_step']*1e3,2), 'us/step host', round(d['host_enqueue_us_per_step'],1), 'mt_mode', d.get('mt_mode'), '| ahead', round(a['gpu_ahead_us_per_step'],2), 'host', round(a['host_enqueue_us_per_step'],1))"
(cd /tmp && timeout -k 10 300 rocprofv3 --hip-runtime-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_emul_api_$TAG -o run -- python3 $ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 > /dev/null 2>$ROOT/gpurun_out/prof_emul_api_$TAG.err) || exit $?
echo done
