# round 4: dense-pass decomposition: micro (dense_parts modes) + product timing-only variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/bin/dense_parts > gpurun_out/dense_parts_r4b.txt 2>&1 || exit $?
cat gpurun_out/dense_parts_r4b.txt
NOTEST=1 bash scripts/gpu_lib_ab.sh r4b base nopull noprep nopart noall
