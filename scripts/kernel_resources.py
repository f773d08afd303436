"""Print VGPR / SGPR / scratch / occupancy per kernel from hipcc's resource remarks.
    python scripts/kernel_resources.py recommendation_gans_amd/csrc/rg_mf.hip [filter] [-DNAME=VAL ...]"""
import re, subprocess, sys
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else ""
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", "include",
                      *defs, "-x", "hip", "-c", src, "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+(.+?): (\S+) \[-Rpass", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
dem = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
for (k, v), name in zip(rows.items(), dem):
    if flt in name:
        print(f"{v.get('VGPRs','?'):>4} vgpr {v.get('AGPRs','?'):>3} agpr {v.get('SGPRs','?'):>4} sgpr "
              f"scratch {v.get('ScratchSize [bytes/lane]','?'):>4} occ {v.get('Occupancy [waves/SIMD]','?'):>2}  {name[:110]}")
