# GPU box: owner-layout parity (world-1 communicator path, world-2 host-staged comm, the DP
# fits), then rank 0 of an 8-rank owner step emulated (plain and under rocprofv3 stats).
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_dp_gpu.py tests/test_dp_fit_gpu.py tests/test_configs_gpu.py -k "dp or owner or rank or Dp or Owner or world" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 > gpurun_out/emul_${TAG}_$k.json 2>gpurun_out/emul_${TAG}_$k.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/emul_${TAG}_$k.json'));print('emul', round(d['ms_per_step']*1e3,2), 'us', round(d['user_update_us'],2), round(d['value']/1e6,1))"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline --dp-at-1 > gpurun_out/dpat1_${TAG}.json 2>gpurun_out/dpat1_${TAG}.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/dpat1_${TAG}.json'));print('dp-at-1', round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e6,1))"
bash scripts/gpu_emul_ab.sh $TAG base
