# GPU box: the gpu test suite (or a subset), then the driver-shaped bench.  Usage: bash scripts/gpu_tests.sh TAG [pytest args]
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "${@:-tests}" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_$TAG.json 2>gpurun_out/bench20_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench20_$TAG.json'));print('b20', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'], d['plan_build_us_per_batch'], d['plan_build_ms_per_epoch'])"
