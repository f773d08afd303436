# GPU box: NCF tests + bench + wave stamps.  Usage: bash scripts/gpu_ncf_wave2.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ncf_gpu.py tests/test_dp_ncf_gpu.py "tests/test_configs_gpu.py::test_ncf_full_size_steps" > gpurun_out/ncfw_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/ncfw_tests_$TAG.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ncf_$TAG.json 2> gpurun_out/bench_ncf_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_ncf_$TAG.json'));r=d.get('roofline') or {};print('ncf', round(d['value']/1e6,3), round(d['ms_per_step'],4), r.get('frac'), r.get('avg_launch_us'))"
timeout -k 10 300 python scripts/ncf_stamps.py --wave --steps 8 > gpurun_out/ncfw_stamps_$TAG.json 2> gpurun_out/ncfw_stamps_$TAG.err || exit $?
cat gpurun_out/ncfw_stamps_$TAG.json
