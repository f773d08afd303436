"""Average of each SQ counter per kernel from scripts/pmc_sq.sh / pmc_gemm.sh.
Usage: python scripts/pmc_sq_summary.py DIR [--per-shape]
--per-shape: group by (kernel, grid size) instead of kernel (one group per GEMM shape)."""
import csv
import glob
import os
import sys
from collections import defaultdict

per_shape = "--per-shape" in sys.argv
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = (row.get("Kernel_Name") or "").replace("(anonymous namespace)::", "")
        name = name.split("(")[0].replace("void ", "").replace("rg::", "")
        if per_shape:
            name += f" grid={row.get('Grid_Size', '?')}"
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in sorted(vals.items()):
    if "gemm" not in name and "rg" not in name and "ncf" not in name and "mf_" not in name and "mt_" not in name:
        continue
    av = {c: sum(v) / len(v) for c, v in cs.items()}
    line = f"{name[:70]:70s}"
    wc = av.get("SQ_WAVE_CYCLES", 0) or 1
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in av:
            line += f" {c[3:]}={av[c] / wc:.2f}"
    if "SQ_LDS_IDX_ACTIVE" in av and av["SQ_LDS_IDX_ACTIVE"]:
        line += f" LDS_CONFLICT/IDX={av.get('SQ_LDS_BANK_CONFLICT', 0) / av['SQ_LDS_IDX_ACTIVE']:.2f}"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in av:
        line += f" MFMA_BUSY={av['SQ_VALU_MFMA_BUSY_CYCLES']:.3g}"
    print(line)
