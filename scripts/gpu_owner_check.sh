# GPU box: the owner-sharded step's tests (world-1 RCCL, world-2 host-staged concurrent step, the
# 8-rank C5 layout) and rank 0 of 8 emulated (scripts/gpu_emul.sh).  Usage: bash scripts/gpu_owner_check.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dp_gpu.py tests/test_configs_gpu.py -k "owner" > gpurun_out/owner_tests_$TAG.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/owner_tests_$TAG.log | tail -20; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_emul.sh $TAG 0
