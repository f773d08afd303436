# A/B of the optimizer-epilogue GEMM variants (RG_GEMM_OPT_STAGES) + cGAN GPU tests under each
set -o pipefail
mkdir -p gpurun_out
for S in ${STAGES:-2 3 4}; do
  RG_GEMM_OPT_STAGES=$S timeout -k 10 120 python scripts/gemm_bench.py --rms-only > gpurun_out/gemm_rms_s$S.jsonl 2>&1 || exit 1
  echo "S=$S"; grep shape gpurun_out/gemm_rms_s$S.jsonl
  RG_GEMM_OPT_STAGES=$S timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gan_gpu.py > gpurun_out/gan_tests_s$S.log 2>&1 || { tail -30 gpurun_out/gan_tests_s$S.log; exit 1; }
  tail -1 gpurun_out/gan_tests_s$S.log
done
