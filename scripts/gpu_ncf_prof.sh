# GPU box: NCF bench + kernel-trace profile (per-kernel stats and the step timeline).  Usage: bash scripts/gpu_ncf_prof.sh TAG [model]
set -o pipefail
TAG=${1:-run}; MODEL=${2:-ncf}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --model $MODEL --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${MODEL}_$TAG.json 2> gpurun_out/bench_${MODEL}_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_${MODEL}_$TAG.json'));r=d.get('roofline') or {};print('$MODEL', round(d['value']/1e6,3), round(d['ms_per_step'],4), r.get('frac'), r.get('avg_launch_us'))"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${MODEL}_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model $MODEL --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_${MODEL}_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_${MODEL}_$TAG.err && echo prof-ok
cd $GRAFT_REPO_ROOT && python scripts/trace_summary.py gpurun_out/prof_${MODEL}_$TAG 2>&1 | tail -40
