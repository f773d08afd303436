# GPU box: the two-launch pipelined MF step -- its bit-identity tests against the split step, the
# MF parity tests (the default path now), then the bench line and a kernel trace of both steps.
# Usage: bash scripts/gpu_pipe2.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_pipe2_gpu.py > gpurun_out/pipe2_tests_$TAG.log 2>&1
rc=$?; echo "pipe2 tests exit=$rc"; tail -3 gpurun_out/pipe2_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for env in "RG_PIPE2=1" "RG_PIPE2=0"; do
  env $env timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pipe2_bench_${TAG}_${env#RG_PIPE2=}.json 2>gpurun_out/pipe2_bench_${TAG}.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/pipe2_bench_${TAG}_${env#RG_PIPE2=}.json'));print('$env', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['kernel'][:40], round(d['roofline']['avg_launch_us'],2))"
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pipe2_prof_$TAG -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/pipe2_prof_$TAG.json 2>$R/gpurun_out/pipe2_prof_$TAG.err) || exit $?
python3 - "$R/gpurun_out/pipe2_prof_$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if n.startswith("void rg::") or n.startswith("rg::"):
            print(n.split("(")[0][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_plan_gpu.py tests/test_claim_gpu.py \
  tests/test_dropin_gpu.py "tests/test_configs_gpu.py::test_mf_full_size_steps" > gpurun_out/pipe2_mftests_$TAG.log 2>&1
rc=$?; echo "mf tests exit=$rc"; tail -3 gpurun_out/pipe2_mftests_$TAG.log
exit $rc
