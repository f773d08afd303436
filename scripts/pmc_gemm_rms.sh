# SQ counters + HBM bytes of the optimizer-epilogue GEMM (gemm_bench.py --rms-only) for
# one RG_GEMM_OPT_STAGES variant.  Usage: bash scripts/pmc_gemm_rms.sh TAG STAGES
set -o pipefail
TAG=${1:-rms}; export RG_GEMM_OPT_STAGES=${2:-7}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcrms_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- \
  python $GRAFT_REPO_ROOT/scripts/gemm_bench.py --rms-only > $OUT/sq.jsonl 2> $OUT/sq.err || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/$C -o run -- \
    python $GRAFT_REPO_ROOT/scripts/gemm_bench.py --rms-only > $OUT/$C.jsonl 2> $OUT/$C.err || exit $?
done
cd $GRAFT_REPO_ROOT && python scripts/pmc_sq_summary.py $OUT/sq --per-shape | tee $OUT/summary.txt
python - "$OUT" <<'PY' | tee -a $OUT/summary.txt
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = defaultdict(list)
    for f in glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm" in r["Kernel_Name"]:
                v[(r["Kernel_Name"].split("(")[0][-40:], r.get("Grid_Size"))].append(float(r["Counter_Value"]))
    for k, x in v.items():
        kib = sum(x) / len(x)
        mb = (2 if c == "FETCH_SIZE" else 1) * kib * 1024 / 1e6
        print(c, k, f"{mb:.1f} MB/launch (corrected)")
PY
