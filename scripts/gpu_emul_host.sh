# GPU box: rank R of an 8-rank owner step emulated on this GPU (bench.py --emulate-rank), with
# the item update all-reduced (RG_OWNER_ITEM_SHARD=0) and sharded (=1): bench line, kernel trace
# stats, and the HIP API trace stats of the host side (where the enqueue time goes).
# Usage: bash scripts/gpu_emul_host.sh TAG [RANK]
set -o pipefail
TAG=${1:-run}
R=${2:-0}
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
for sh in 0 1; do
  T=${TAG}_is$sh
  RG_OWNER_ITEM_SHARD=$sh timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank $R/8 > gpurun_out/emul_$T.json 2>gpurun_out/emul_$T.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/emul_$T.json'));print('emul $T', round(d['ms_per_step']*1e3,2), 'us/step; user update', round(d['user_update_us'],2), 'host enqueue', round(d['host_enqueue_us_per_step'],2))"
  (cd /tmp && RG_OWNER_ITEM_SHARD=$sh timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_emul_$T -o run -- python3 $ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank $R/8 > $ROOT/gpurun_out/prof_emul_bench_$T.json 2>$ROOT/gpurun_out/prof_emul_$T.err) || exit $?
done
[ -n "$API" ] || { echo done; exit 0; }
T=${TAG}_is0
(cd /tmp && RG_OWNER_ITEM_SHARD=0 timeout -k 10 300 rocprofv3 --hip-runtime-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_emul_api_$T -o run -- python3 $ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank $R/8 > $ROOT/gpurun_out/prof_emul_api_bench_$T.json 2>$ROOT/gpurun_out/prof_emul_api_$T.err) || exit $?
echo done
