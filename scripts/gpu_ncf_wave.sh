# GPU box: NCF tests (wave kernel for E = 64) + NCF bench, new vs tile kernel (RG_NCF_TILE=1).
# Usage: bash scripts/gpu_ncf_wave.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ncf_gpu.py tests/test_dp_ncf_gpu.py tests/test_dp_ncf_fit_gpu.py "tests/test_configs_gpu.py::test_ncf_full_size_steps" \
  tests/test_dropin_gpu.py > gpurun_out/ncfw_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/ncfw_tests_$TAG.log | tail -15
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  RG_NCF_TILE=$v timeout -k 10 300 python3 bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ncf_t${v}_$TAG.json 2> gpurun_out/bench_ncf_t${v}_$TAG.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_ncf_t${v}_$TAG.json'));r=d.get('roofline') or {};print('tile=$v', round(d['value']/1e6,3), round(d['ms_per_step'],4), r.get('frac'), r.get('avg_launch_us'))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_ncf_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG.err && echo prof-ok
