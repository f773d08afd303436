# GPU box: full gpu tests, smoke, driver-exact bench (x3), long bench, kernel-trace stats.
# Usage: bash scripts/gpu_r2.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
echo smoke-ok
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_${TAG}_$k.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench20_${TAG}_$k.json'));print('b20', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench200_$TAG.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench200_$TAG.json'));print('b200', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.err && echo prof-ok
