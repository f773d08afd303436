"""Per-kernel HBM traffic from the two rocprofv3 --pmc passes of scripts/pmc_apply.sh.

bytes/launch = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE, averaged over launches:
FETCH_SIZE/WRITE_SIZE are in KiB, and on gfx950 FETCH_SIZE counts exactly half of
the bytes of wide (16 B/lane) coalesced streaming reads (MI355X_MICROARCH.md, HBM).
Writes profiles/pmc_step.json (overlapped step: front + hot kernels) or
profiles/pmc_apply.json (split step: rg_mf_apply) when --write is given; bench.py
reads it as roofline.traffic."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(path):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
            v = row.get("Counter_Value") or row.get("Counter-Value")
            if v is None:
                continue
            vals[name].append(float(v))
    return vals


def short(name):
    for key in ("mf_apply_kernel", "mf_pairs_kernel", "mt_generate_kernel", "mf_prepare_kernel", "mf_front_kernel",
                "mf_hot_kernel", "mt_head_kernel", "mt_jump_kernel", "mt_tail_kernel", "mf_back_kernel"):
        if key in name:
            return key
    return None


def main():
    root = sys.argv[1]
    fetch, write = per_kernel(os.path.join(root, "FETCH_SIZE")), per_kernel(os.path.join(root, "WRITE_SIZE"))
    out = {}
    for name in set(fetch) | set(write):
        k = short(name)
        if k is None:
            continue
        f = sum(fetch.get(name, [0])) / max(len(fetch.get(name, [])), 1)
        w = sum(write.get(name, [0])) / max(len(write.get(name, [])), 1)
        out.setdefault(k, {}).update({"kernel": name[:120], "fetch_kib_raw": f, "write_kib": w,
                                      "launches": len(fetch.get(name, [])),
                                      "hbm_bytes_per_launch": 2 * 1024 * f + 1024 * w})
    bench = os.path.join(root, "bench_FETCH_SIZE.json")
    cfg = json.load(open(bench)) if os.path.exists(bench) else {}
    import hashlib
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "recommendation_gans_amd",
                       "librg_hip.so")
    res = {"source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 20",
           "lib_sha16": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16],
           "dim": cfg.get("config", {}).get("embedding_dim"), "batch": cfg.get("config", {}).get("global_batch"),
           "kernels": out}
    name = "pmc_apply.json"
    if "mf_apply_kernel" in out:
        res["hbm_bytes_per_launch"] = out["mf_apply_kernel"]["hbm_bytes_per_launch"]
    if "mf_back_kernel" in out:       # split step: rg_mf_apply_prepare
        res["hbm_bytes_per_launch"] = out["mf_back_kernel"]["hbm_bytes_per_launch"]
        name = "pmc_back.json"
    if "mf_front_kernel" in out and "mf_hot_kernel" in out:     # overlapped step: one of each per step
        res["hbm_bytes_per_step"] = (out["mf_front_kernel"]["hbm_bytes_per_launch"] +
                                     out["mf_hot_kernel"]["hbm_bytes_per_launch"])
        name = "pmc_step.json"
    print(json.dumps(res, indent=1))
    if "--write" in sys.argv:
        json.dump(res, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                                         name), "w"), indent=1)


if __name__ == "__main__":
    main()
