# GPU box: MF parity tests (fused + split), bench, kernel-trace stats.  Usage: bash scripts/gpu_mf.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_dp_gpu.py ${K:+-k "$K"} > gpurun_out/mf_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 gpurun_out/mf_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-baseline-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
echo bench-ok && cat gpurun_out/bench_$TAG.json
RG_FUSED=0 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_split_$TAG.json 2> gpurun_out/bench_split_$TAG.err || exit $?
echo split-ok && cat gpurun_out/bench_split_$TAG.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.err && echo prof-ok
