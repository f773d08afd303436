# NCF on the GPU box: parity tests, bench line, kernel-trace profile.  Usage: bash scripts/ncf_check.sh TAG
set -o pipefail
TAG=${1:-ncf}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_ncf_gpu.py -q -p no:cacheprovider > gpurun_out/ncf_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/ncf_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --model ncf --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_ncf_$TAG.json 2> gpurun_out/bench_ncf_$TAG.err || exit $?
echo bench-ok && cat gpurun_out/bench_ncf_$TAG.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --model ncf --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_ncf_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG.err && echo prof-ok
python $GRAFT_REPO_ROOT/scripts/trace_summary.py $GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG 2>/dev/null | head -30 || true
