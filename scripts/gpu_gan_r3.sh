# GPU box: the persistent staggered optimizer GEMM -- bitwise vs the one-tile kernel, the cGAN parity tests,
# then the C4 bench A/B (RG_GEMM_OPT_PERSIST 0/1) and a kernel-stats profile.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gan_gpu.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for p in 0 1; do
    RG_GEMM_OPT_PERSIST=$p timeout -k 10 300 python3 bench.py --model gan --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/gan_${TAG}_p${p}_$k.json 2>gpurun_out/gan_${TAG}_p${p}_$k.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/gan_${TAG}_p${p}_$k.json'));print('persist=$p', round(d['value'],1), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],4))"
  done
done
for sg in 0 1500 6000; do
  RG_GEMM_STAGGER_NS=$sg timeout -k 10 300 python3 bench.py --model gan --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/gan_${TAG}_sg$sg.json 2>gpurun_out/gan_${TAG}_sg$sg.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/gan_${TAG}_sg$sg.json'));print('stagger=$sg', round(d['value'],1), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],4))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ganprof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model gan --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/ganprof_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/ganprof_$TAG.err && echo prof-ok
