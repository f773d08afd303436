# cGAN on the GPU box: GEMM + step parity tests.  Usage: bash scripts/gan_check.sh TAG
set -o pipefail
TAG=${1:-gan}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gan_gpu.py -q -x -p no:cacheprovider > gpurun_out/gan_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -30 gpurun_out/gan_tests_$TAG.log
exit $rc
