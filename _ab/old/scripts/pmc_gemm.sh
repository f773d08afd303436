# SQ counters of the cGAN GEMM shapes (scripts/gemm_bench.py).  Usage: bash scripts/pmc_gemm.sh TAG
set -o pipefail
TAG=${1:-gemm}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcgemm_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python scripts/gemm_bench.py > $OUT/bench.jsonl 2>$OUT/bench.err || exit $?
cat $OUT/bench.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT -o run -- \
  python $GRAFT_REPO_ROOT/scripts/gemm_bench.py > $OUT/prof.jsonl 2> $OUT/prof.err || exit $?
cd $GRAFT_REPO_ROOT && python scripts/pmc_sq_summary.py $OUT --per-shape | tee $OUT/summary.txt
