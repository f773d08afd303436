# GPU box: the NCF / NeuMF GPU tests, then the NCF and NeuMF bench lines and a kernel-stats
# profile of the NCF step.  Usage: bash scripts/gpu_ncf.sh TAG
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ncf_wave_gpu.py tests/test_ncf_gpu.py > gpurun_out/ncf_tests_$TAG.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/ncf_tests_$TAG.log | tail -40; [ $rc -eq 0 ] || exit $rc
for m in ncf neumf; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${m}_$TAG.json 2> gpurun_out/bench_${m}_$TAG.err || { tail -5 gpurun_out/bench_${m}_$TAG.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${m}_$TAG.json')); r=d['roofline']; print('$m', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step;', r['kernel'], round(r['avg_launch_us'],1), 'us', round(r['frac'],3))"
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ncf_prof_$TAG -o run -- python3 $R/bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > $R/gpurun_out/ncf_prof_$TAG.json 2>$R/gpurun_out/ncf_prof_$TAG.err) || exit $?
python3 - "$R/gpurun_out/ncf_prof_$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"].split("(")[0][-60:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
