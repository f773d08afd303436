# GPU box: NCF bench line + the wave kernel's rocprof average per library variant (timing only:
# no tests -- RG_X_ variants compute wrong results on purpose).  Usage: bash scripts/gpu_ncf_var.sh TAG variant...
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/recommendation_gans_amd/librg_hip.so
  [ $v = base ] || lib=$R/recommendation_gans_amd/_variants/librg_hip_$v.so
  (cd /tmp && RG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ncfvar_prof_${v}_$TAG -o run -- python3 $R/bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > $R/gpurun_out/ncfvar_${v}_$TAG.json 2>$R/gpurun_out/ncfvar_${v}_$TAG.err) || exit 1
  python3 - "$R/gpurun_out/ncfvar_prof_${v}_$TAG" "$v" <<'PY'
import csv, glob, sys
k = [r for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(f))
     if "ncf_wave_kernel" in r["Name"] or "mf_back_kernel" in r["Name"]]
print(sys.argv[2], "; ".join(f"{r['Name'].split('(')[0][-40:]} {round(float(r['AverageNs']) / 1e3, 2)} us" for r in k))
PY
done
