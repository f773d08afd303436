# GPU box: the data-parallel MF tests (owner-sharded, replicated, user-sharded layouts; C5 at
# 8 ranks on one GPU) against the product library.  Usage: bash scripts/gpu_dp_check.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dp_gpu.py tests/test_dp_fit_gpu.py "tests/test_configs_gpu.py::test_mf_owner_full_size_8_ranks_d128" \
  "tests/test_configs_gpu.py::test_mf_dp_rank_gradient_d128" > gpurun_out/dpcheck_tests_$TAG.log 2>&1
rc=$?; echo "dp tests exit=$rc"; tail -3 gpurun_out/dpcheck_tests_$TAG.log
exit $rc
