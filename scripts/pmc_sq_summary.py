"""Average of each SQ counter per kernel from scripts/pmc_sq.sh.  Usage: python scripts/pmc_sq_summary.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = (row.get("Kernel_Name") or "").split("(")[0].replace("void ", "").replace("rg::", "")
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in sorted(vals.items()):
    if "rg" not in name and "ncf" not in name and "mf_" not in name and "mt_" not in name:
        continue
    print(name[:60])
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}")
