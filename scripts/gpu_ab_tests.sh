# GPU box: the tests of the measured-slower alternatives (lazy dense pass, overlapped step,
# pipelined steps, the owner step's sharded item update and MT rank slices, the wave-specialised optimizer GEMM: tests/test_gan_gpu.py),
# which only the A/B build carries.  Build it here first:
#   python -m recommendation_gans_amd.build --variant ab -DRG_AB=1
set -o pipefail
mkdir -p gpurun_out
RG_LIB=recommendation_gans_amd/_variants/librg_hip_ab.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider -m gpu tests/test_lazy_gpu.py tests/test_mf_fused_gpu.py tests/test_pipe_gpu.py \
  tests/test_pipe2_gpu.py tests/test_gan_gpu.py "tests/test_dp_gpu.py::test_owner_native_concurrent_step_world2" \
  tests/test_dp_gpu.py::test_owner_mt_slices_match_the_full_walk \
  > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -20 gpurun_out/ab_tests.log; exit $rc
