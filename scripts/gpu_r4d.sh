# round 4: same-box isolation of the dense pass: micro floor vs product variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/bin/dense_floor > gpurun_out/dense_floor_r4d.txt 2>&1 || exit $?
head -7 gpurun_out/dense_floor_r4d.txt
NOTEST=1 bash scripts/gpu_lib_ab.sh r4d base lean so sonp
