# GPU box: MF tests, decomposition of the step (scripts/mf_step_probe.py, one rocprof pass per
# variant) and bench variants.  Usage: bash scripts/gpu_probe.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out/probe_$TAG
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_dp_gpu.py > gpurun_out/mf_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -2 gpurun_out/mf_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in split fused_scan fused_owner front_pairs_only two_stream serial; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/probe_$TAG/$v -o run -- python $R/scripts/mf_step_probe.py --variant $v --iters 40 > $R/gpurun_out/probe_$TAG/$v.txt 2>&1) || exit $?
  echo "== $v: $(grep '^'$v' ' gpurun_out/probe_$TAG/$v.txt)"
  python - "gpurun_out/probe_$TAG/$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "rg::" in n and "mt_" not in n:
        print(f'   {r["Calls"]:>4} {float(r["AverageNs"])/1000:7.1f}us {n.split("(")[0][:70]}')
PY
done
for cfg in "RG_X=0" "RG_APPLY_SPEC=1" "RG_APPLY_NT=1" "RG_APPLY_SPEC=1 RG_APPLY_NT=1" "RG_MT_UNITS=1" "RG_FUSED=1" "RG_FUSED=1 RG_HOT_SCAN=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b_$TAG.json 2>/dev/null || exit $?
  echo "$cfg" $(tail -1 gpurun_out/b_$TAG.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; ev', round(d['roofline']['avg_launch_us'],1), 'us; host', round(d['host_enqueue_us_per_step'],1))")
done
