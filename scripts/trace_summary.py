"""Per-kernel durations and same-queue gaps of the last steps of a rocprofv3
--kernel-trace run (rg kernels only).  Usage: python scripts/trace_summary.py DIR"""
import csv
import glob
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "rg::" in r["Kernel_Name"]]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("<")[0].split("(")[0]
             .replace("void ", "").replace("rg::", ""), r["Queue_Id"]) for r in rows)
ks = ks[len(ks) // 2:]                      # steady state: second half
dur = defaultdict(list)
gaps = defaultdict(list)
last_end = {}
for s, e, n, q in ks:
    dur[n].append((e - s) / 1e3)
    if q in last_end:
        gaps[n].append((s - last_end[q]) / 1e3)
    last_end[q] = e
span = (ks[-1][1] - ks[0][0]) / 1e3
npairs = len(dur.get("mf_pairs_kernel") or dur.get("owner_scores_kernel") or dur.get("ncf_wave_kernel") or dur.get("ncf_pairs_kernel") or [1])
print(sys.argv[1], f"span/step {span / npairs:.1f} us")
for n in dur:
    d, g = dur[n], gaps.get(n, [0])
    print(f"  {n:22s} n={len(d):4d} dur {sum(d) / len(d):6.1f} us   gap-before {sum(g) / len(g):6.1f} us")
