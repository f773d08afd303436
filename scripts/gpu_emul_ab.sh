# GPU box: rank R of an 8-rank owner step emulated on this GPU (bench.py --emulate-rank) under
# rocprofv3 kernel-trace stats, for each library variant (base = the product library; timing-only
# variants from python -m recommendation_gans_amd.build --variant NAME -DRG_X_...).
# Usage: bash scripts/gpu_emul_ab.sh TAG base nopart ...
set -o pipefail
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for name in "$@"; do
  if [ "$name" = base ]; then lib=$R/recommendation_gans_amd/librg_hip.so
  else lib=$R/recommendation_gans_amd/_variants/librg_hip_$name.so; fi
  (cd /tmp && RG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/emulab_${TAG}_$name -o run -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --emulate-rank 0/8 > $R/gpurun_out/emulab_${TAG}_$name.json 2>$R/gpurun_out/emulab_${TAG}_$name.err) || exit $?
  python3 - "$R/gpurun_out/emulab_${TAG}_$name" "$name" "$R/gpurun_out/emulab_${TAG}_$name.json" <<'PY'
import csv, glob, json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[2], "step_us", round(d["ms_per_step"] * 1e3, 2))
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if int(r["Calls"]) >= 50:
            print("   ", r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:95])
PY
done
