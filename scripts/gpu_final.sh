# GPU box, end of round: every gpu test + smoke + driver-shaped benches + kernel-trace profiles
# (scripts/gpu_full.sh), the PMC traffic of the dense pass (scripts/pmc_apply.sh), then every
# bench mode (scripts/gpu_benches.sh).  Usage: bash scripts/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
bash scripts/gpu_full.sh $TAG || exit $?
bash scripts/pmc_apply.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
echo pmc-ok
bash scripts/gpu_benches.sh $TAG || exit $?
