# cGAN bench line + kernel-trace profile.  Usage: bash scripts/gan_bench.sh TAG
set -o pipefail
TAG=${1:-gan}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model gan --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_gan_$TAG.json 2> gpurun_out/bench_gan_$TAG.err || { tail -20 gpurun_out/bench_gan_$TAG.err; exit 1; }
echo bench-ok && cat gpurun_out/bench_gan_$TAG.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_gan_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --model gan --steps 25 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_gan_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_gan_$TAG.err && echo prof-ok
head -30 $GRAFT_REPO_ROOT/gpurun_out/prof_gan_$TAG/run_kernel_stats.csv | cut -c1-220
