# GPU box: a pytest subset (first arg: tag, rest: files / -k), with RG_REPORT_DIR reports under gpurun_out/.
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out/reports_$TAG
export TMPDIR=/tmp RG_REPORT_DIR=$GRAFT_REPO_ROOT/gpurun_out/reports_$TAG
timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -30
exit $rc
