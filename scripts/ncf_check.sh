# NCF on the GPU box: parity tests, bench lines (NCF, NeuMF), kernel-trace profile.  Usage: bash scripts/ncf_check.sh TAG
set -o pipefail
TAG=${1:-ncf}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ncf_gpu.py tests/test_neumf_gpu.py tests/test_dp_ncf_gpu.py -p no:cacheprovider > gpurun_out/ncf_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/ncf_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/ncf_tests_$TAG.log
for M in ncf neumf; do
  timeout -k 10 300 python bench.py --model $M --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_${M}_$TAG.json 2> gpurun_out/bench_${M}_$TAG.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_${M}_$TAG.json'));print('$M', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], d['roofline'].get('frac'))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --model ncf --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench_ncf_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG.err && echo prof-ok
head -6 $GRAFT_REPO_ROOT/gpurun_out/prof_ncf_$TAG/run_kernel_stats.csv | cut -c1-160
