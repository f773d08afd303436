# GPU box: the NCF tail's dense pass on the 8-lane x 2-float4 row layout (product) against the
# 16-lane layout (variant ncfold): NCF / NeuMF GPU tests on the product, then per library an NCF
# bench line and its kernel stats.  Usage: bash scripts/gpu_ncf_v.sh TAG
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ncf_wave_gpu.py tests/test_ncf_gpu.py tests/test_neumf_gpu.py > gpurun_out/ncfv_tests_$TAG.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/ncfv_tests_$TAG.log | tail -3; [ $rc -eq 0 ] || exit $rc
for v in base ncfold; do
  lib=$R/recommendation_gans_amd/librg_hip.so
  [ $v = base ] || lib=$R/recommendation_gans_amd/_variants/librg_hip_$v.so
  for m in ncf neumf; do
    RG_LIB=$lib timeout -k 10 300 python3 bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ncfv_${m}_${v}_$TAG.json 2>gpurun_out/ncfv_${m}_${v}_$TAG.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ncfv_${m}_${v}_$TAG.json')); print('$v $m', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  done
  (cd /tmp && RG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ncfv_prof_${v}_$TAG -o run -- python3 $R/bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > /dev/null 2>$R/gpurun_out/ncfv_prof_${v}_$TAG.err) || exit 1
  python3 - "$R/gpurun_out/ncfv_prof_${v}_$TAG" "$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rg::" in r["Name"]:
            print(sys.argv[2], r["Name"].split("(")[0][-70:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
