# GPU box: MF parity tests, then bench at the driver's 20/5 and at 200/20 for env variants.
# Usage: bash scripts/gpu_bench_ab.sh TAG "name1:ENV=1 ENV2=0" "name2:..."   (tests skipped if NOTEST=1)
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_dropin_gpu.py ${TESTS:-} > gpurun_out/ab_tests_$TAG.log 2>&1
  rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/ab_tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  for st in "20 5" "200 20"; do
    set -- $st
    env $envs timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${TAG}_${name}_$1.json 2>gpurun_out/ab_${TAG}_${name}_$1.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_${name}_$1.json'));print('$name', $1, round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2))"
  done
done
