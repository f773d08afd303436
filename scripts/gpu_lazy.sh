# GPU box: lazy-pass parity tests (+ the MF / drop-in suites), then the driver-shaped bench
# lazy and eager (RG_LAZY=0) on the same box.  Usage: bash scripts/gpu_lazy.sh TAG [pytest files]
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider ${@:-tests/test_lazy_gpu.py} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_${TAG}_$k.json 2>gpurun_out/bench20_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench20_${TAG}_$k.json'));print('lazy b20', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('lazy_dense_pass',{}).get('user_rows_per_step'))"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench200_$TAG.json 2>>gpurun_out/bench20_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench200_$TAG.json'));print('lazy b200', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'])"
RG_LAZY=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_eager_$TAG.json 2>>gpurun_out/bench20_$TAG.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench20_eager_$TAG.json'));print('eager b20', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_us'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.err && echo prof-ok
