# round 4: lean pull (register-light dense pass) A/B; parity tests on the lean library first
set -o pipefail
mkdir -p gpurun_out
RG_LIB=$GRAFT_REPO_ROOT/recommendation_gans_amd/_variants/librg_hip_lean.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_plan_gpu.py tests/test_claim_gpu.py > gpurun_out/r4c_tests_lean.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_tests_lean.log; [ $rc -eq 0 ] || exit $rc
NOTEST=1 bash scripts/gpu_lib_ab.sh r4c base lean lean4 leannofix
