# GPU box: every gpu test, smoke, the driver-shaped bench, the owner-path bench, kernel-trace profiles of both.
# Usage: bash scripts/gpu_full.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -4 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
echo smoke-ok
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_$TAG.json 2>gpurun_out/bench20_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench20_$TAG.json'));print('b20', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'], d['plan_build_us_per_batch'])"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 5 --no-cpu-baseline --dp owner --dp-at-1 > gpurun_out/bench_own_$TAG.json 2>gpurun_out/bench_own_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_own_$TAG.json'));print('own', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_own_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --dp owner --dp-at-1 > $GRAFT_REPO_ROOT/gpurun_out/prof_own_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_own_$TAG.err && echo prof-ok
