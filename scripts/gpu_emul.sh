# GPU box: the driver-shaped 1-GPU bench, then rank R of an 8-rank owner step emulated on
# this GPU (bench.py --emulate-rank), plain and under rocprofv3 kernel-trace stats.
# Usage: bash scripts/gpu_emul.sh TAG [RANK]
set -o pipefail
TAG=${1:-run}
R=${2:-0}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_$TAG.json 2>gpurun_out/bench20_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench20_$TAG.json'));print('b20', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'])"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank $R/8 > gpurun_out/emul_$TAG.json 2>gpurun_out/emul_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/emul_$TAG.json'));print('emul', d['ms_per_step'], d['user_update_us'], d['value']/1e6)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_emul_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank $R/8 > $GRAFT_REPO_ROOT/gpurun_out/prof_emul_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_emul_$TAG.err && echo prof-ok
