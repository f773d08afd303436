# GPU box: same-box A/B of the MF bench, previous build (_ab/old) vs this tree, interleaved,
# then a kernel trace of this tree's bench.  Usage: bash scripts/gpu_ab.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_dp_gpu.py tests/test_dropin_gpu.py tests/test_ncf_gpu.py > gpurun_out/ab_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -2 gpurun_out/ab_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/mf_pairs_stamps.py --steps 20 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('stamps', d['span_us'], d['phase_median_us'], d['ids_phase_us_by_start_quartile'])" || exit $?
run() {  # dir label env...
  local d=$1 l=$2; shift 2
  (cd $d && env "$@" timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > $R/gpurun_out/ab_$TAG.json 2>/dev/null) || return $?
  echo "$l" $(tail -1 gpurun_out/ab_$TAG.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; ev', round(d['roofline']['avg_launch_us'],1), 'us; host', round(d['host_enqueue_us_per_step'],1))")
}
for k in 1 2; do
  run $R/abold old RG_X=0 || exit $?
  run $R new RG_X=0 || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $R/gpurun_out/prof_bench_$TAG.json 2>$R/gpurun_out/prof_$TAG.err && echo prof-ok
