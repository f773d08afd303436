# GPU box: NCF tests with the current library, then NCF bench A/B against a base library
# (RG_LIB=_variants/librg_hip_base.so), alternating.  Usage: bash scripts/gpu_ncf_ab.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ncf_gpu.py tests/test_dp_ncf_gpu.py "tests/test_configs_gpu.py::test_ncf_full_size_steps" > gpurun_out/ncfab_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -2 gpurun_out/ncfab_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export RG_LIB=$PWD/recommendation_gans_amd/_variants/librg_hip_base.so; else unset RG_LIB; fi
    timeout -k 10 300 python3 bench.py --model ncf --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ncfab_${v}${k}_$TAG.json 2> gpurun_out/ncfab_${v}${k}_$TAG.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ncfab_${v}${k}_$TAG.json'));r=d.get('roofline') or {};print('$v$k', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1), r.get('avg_launch_us'))"
  done
done
