# GPU box: NCF / NeuMF tests, then bench + trace with the inline prefetch vs the side-stream one.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ncf_gpu.py tests/test_neumf_gpu.py tests/test_dp_ncf_gpu.py tests/test_dp_ncf_fit_gpu.py > gpurun_out/ncfpf_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/ncfpf_tests_$TAG.log | tail -15
[ $rc -eq 0 ] || exit $rc
for side in 0 1; do export RG_NCF_GEN_INLINE=$side;
  for m in ncf neumf; do
    timeout -k 10 300 python3 bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${m}_s${side}_$TAG.json 2> gpurun_out/bench_${m}_s${side}_$TAG.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/bench_${m}_s${side}_$TAG.json'));r=d.get('roofline') or {};print('$m geninline=$side', round(d['value']/1e6,3), round(d['ms_per_step'],4), r.get('frac'), r.get('avg_launch_us'))"
  done
done
unset RG_NCF_GEN_INLINE; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ncfpf_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_ncfpf_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_ncfpf_$TAG.err && echo prof-ok
cd $GRAFT_REPO_ROOT && python scripts/trace_summary.py gpurun_out/prof_ncfpf_$TAG 2>&1 | tail -10
