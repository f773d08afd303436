# cGAN tests, then bench + profile.  Usage: bash scripts/gan_all.sh TAG
set -o pipefail
TAG=${1:-gan}
bash scripts/gan_check.sh $TAG && bash scripts/gan_bench.sh $TAG && python scripts/trace_summary.py gpurun_out/prof_gan_$TAG 2>/dev/null | head -40
