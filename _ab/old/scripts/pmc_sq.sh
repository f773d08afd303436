# SQ counters (one pass) per kernel for a bench model: wave cycles split into
# parked / issue-stalled / active, LDS conflicts, MFMA busy.
# Usage: bash scripts/pmc_sq.sh TAG [mf|ncf]   -> gpurun_out/pmcsq_TAG/
set -o pipefail
TAG=${1:-run}; MODEL=${2:-ncf}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcsq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --model $MODEL --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
cd $GRAFT_REPO_ROOT && python scripts/pmc_sq_summary.py $OUT | tee $OUT/summary.txt
