# GPU box: lazy-pass parity (both load orders), then timing A/B of the variants vs eager.
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_lazy_gpu.py > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
RG_LAZY_SPEC=1 RG_LAZY_CAP=2 timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_lazy_gpu.py > gpurun_out/gpu_tests_spec_$TAG.log 2>&1 || { echo "spec tests failed"; tail -30 gpurun_out/gpu_tests_spec_$TAG.log; exit 1; }
echo tests-ok
for v in "RG_LAZY_SPEC=0" "RG_LAZY_SPEC=1" "RG_LAZY_SPEC=1 RG_LAZY_CAP=2" "RG_LAZY_SPEC=1 RG_LAZY_CAP=1" "RG_LAZY_SPEC=1 RG_LAZY_DBG=1" "RG_LAZY=0"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $v timeout -k 10 300 python3 bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_${TAG}_$tag.json 2>>gpurun_out/b_$TAG.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_$tag.json'));print('$v', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d.get('lazy_dense_pass',{}).get('user_rows_per_step'))"
done
