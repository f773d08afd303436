# GPU box: same-box A/B of the E = 64 NCF wave kernel's tile height (32 rows: the product; 48
# rows: variant ncf48, -DRG_NCF_WAVE_ROWS=48), interleaved, with the NCF tests against the
# 48-row build first.  Build the variant here first (it is not kept in the tree):
#   python -m recommendation_gans_amd.build --variant ncf48 -DRG_NCF_WAVE_ROWS=48
set -o pipefail
mkdir -p gpurun_out
RG_LIB=recommendation_gans_amd/_variants/librg_hip_ncf48.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider -m gpu tests/test_ncf_wave_gpu.py > gpurun_out/ncf48_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ncf48_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in "r32|" "r48|recommendation_gans_amd/_variants/librg_hip_ncf48.so"; do
    IFS='|' read name lib <<< "$cfg"
    env ${lib:+RG_LIB=$lib} timeout -k 10 300 python bench.py --model ncf --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/nab.json 2>gpurun_out/nab.err || { tail -3 gpurun_out/nab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/nab.json')); r=d['roofline']; print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; pair kernel', round(r['avg_launch_us'],1), 'us', round(r['frac'],3))"
  done
done
