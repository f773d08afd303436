# HBM traffic of the bench kernels from PMC counters, one counter per pass (gfx950:
# FETCH_SIZE and WRITE_SIZE do not fit one pass), kernel trace only (no sys/runtime
# trace with --pmc).  Usage: bash scripts/pmc_apply.sh TAG   -> gpurun_out/pmc_TAG/
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/$C -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || exit $?
done
cd $GRAFT_REPO_ROOT && python scripts/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG/summary.json && cat gpurun_out/pmc_$TAG/summary.json
