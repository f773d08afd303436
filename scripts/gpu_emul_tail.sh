# GPU box: rank 0 of 8 emulated with the jump-ahead MT walk split into N tail segments per ring
# slot (RG_MT_TAIL, A/B build): fewer segments = less jump work on every CU, longer walks on fewer.
# Usage: bash scripts/gpu_emul_tail.sh TAG N...
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
AB=$GRAFT_REPO_ROOT/recommendation_gans_amd/_variants/librg_hip_ab.so
for t in "$@"; do
  RG_LIB=$AB RG_MT_TAIL=$t timeout -k 10 300 python3 bench.py --gpus 1 --steps 64 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 > gpurun_out/emul_tail_${TAG}_$t.json 2>gpurun_out/emul_tail_${TAG}_$t.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/emul_tail_${TAG}_$t.json'));print('tail $t', round(d['ms_per_step']*1e3,2), 'us/step; host', round(d['host_enqueue_us_per_step'],1))"
done
