# GPU box: the MF parity tests against the product library (or RG_LIB), then the dense-pass
# attribution variants (scripts/gpu_attr.sh).  Usage: bash scripts/gpu_mf_check.sh TAG [attr names...]
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_plan_gpu.py tests/test_claim_gpu.py \
  "tests/test_configs_gpu.py::test_mf_full_size_steps" > gpurun_out/mfcheck_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/mfcheck_tests_$TAG.log; grep -E "PASSED|FAILED" gpurun_out/mfcheck_tests_$TAG.log | grep -c PASSED
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/parity_elementwise.jsonl gpurun_out/parity_mf_$TAG.jsonl 2>/dev/null
[ $# -gt 0 ] && bash scripts/gpu_attr.sh $TAG "$@"
exit 0
