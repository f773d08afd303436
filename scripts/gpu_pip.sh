# GPU box: the next step's prepare in the pair pass (RG_PREP_IN_PAIRS=1) -- MF parity tests
# under it, then a same-box bench A/B against the prepare in the dense pass.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
RG_PREP_IN_PAIRS=1 timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_claim_gpu.py tests/test_mf_gpu.py tests/test_dropin_gpu.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -2 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_env.sh $TAG "RG_PREP_IN_PAIRS=0" "RG_PREP_IN_PAIRS=1" -- --steps 200 --warmup 20
