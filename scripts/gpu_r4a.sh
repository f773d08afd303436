# round 4: dense-pass floor micro + write-through store A/B of the product step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/bin/dense_floor > gpurun_out/dense_floor_r4a.txt 2>&1 || exit $?
cat gpurun_out/dense_floor_r4a.txt
NOTEST=1 bash scripts/gpu_lib_ab.sh r4a base wt
