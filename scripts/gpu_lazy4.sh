# GPU box: lazy-pass parity, then timing A/B (product, no-catch-up experiment, eager).
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider ${@:-tests/test_lazy_gpu.py} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
for v in "RG_LAZY_DBG=0" "RG_LAZY_DBG=1" "RG_LAZY_SPEC=1" "RG_LAZY=0"; do
  env $v timeout -k 10 300 python3 bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_${TAG}_${v}.json 2>>gpurun_out/b_$TAG.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d.get('lazy_dense_pass',{}).get('user_rows_per_step'))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.err && echo prof-ok
