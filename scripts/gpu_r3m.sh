# GPU box: drop-in no-negatives fit test, lazy-pass timing experiments, a HIP API trace of the cGAN bench.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_dropin_gpu.py tests/test_lazy_gpu.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
bash scripts/gpu_lazy6.sh $TAG || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gantrace_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model gan --steps 10 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/gantrace_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/gantrace_$TAG.err && echo gantrace-ok
