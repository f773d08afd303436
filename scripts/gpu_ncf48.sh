# GPU box: the NCF tests with the product's 48-row wave tiles (every NCF / NeuMF / NCF-DP GPU test
# and C3's 10 full-size steps), then NCF bench lines of the product and the 32-row variant
# (ncf32), interleaved twice.  Usage: bash scripts/gpu_ncf48.sh TAG
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ncf_wave_gpu.py tests/test_ncf_gpu.py tests/test_neumf_gpu.py tests/test_dp_ncf_gpu.py \
  tests/test_dp_ncf_fit_gpu.py tests/test_configs_gpu.py -k "ncf or neumf or NCF" > gpurun_out/ncf48_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/ncf48_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in base ncf32; do
  lib=$R/recommendation_gans_amd/librg_hip.so
  [ $v = base ] || lib=$R/recommendation_gans_amd/_variants/librg_hip_$v.so
  RG_LIB=$lib timeout -k 10 300 python3 bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ncf48_${v}_${rep}_$TAG.json 2>gpurun_out/ncf48_${v}_${rep}_$TAG.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ncf48_${v}_${rep}_$TAG.json')); r=d['roofline']; print('$v rep $rep', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step', round(r['avg_launch_us'],1), 'us', round(r['frac'],3))"
done; done
