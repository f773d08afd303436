# GPU box check: parity tests, smoke, bench, kernel-trace profile.  Usage: bash scripts/gpu_check.sh TAG
# Plain test failures (exit 1) continue to the next step; a crash, abort or time limit ends the script.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] && echo smoke-ok || tail -3 gpurun_out/smoke_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-baseline-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
echo bench-ok && cat gpurun_out/bench_$TAG.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.err && echo prof-ok
