# GPU box: attribution of the MF dense pass (mf_back_kernel) by timing-only library variants
# (build.py --variant NAME --only rg_mf.hip -DRG_X_...: round 6 removed the RG_X_ blocks from the
# sources, their results are under profiles/ and the code in the history; results of X variants are wrong, the
# timings are what they are for).  Per variant: a 20-step bench line and a 50-step rocprofv3
# kernel trace (average mf_back / mf_pairs / mf_prepare durations).
# Usage: bash scripts/gpu_attr.sh TAG name[:ENV=VAL] ...   (base* = the product library; a variant
# name's part before '+' names the library; BARGS=... in the ENV part: extra bench.py arguments,
# e.g. v16:BARGS=--dim=128)
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=gpurun_out/attr_$TAG.txt
for spec in "$@"; do
  name=${spec%%:*}; envs=""; [ "$name" != "$spec" ] && envs=${spec#*:}
  lib=$R/recommendation_gans_amd/librg_hip.so
  case $name in base*) ;; *) lib=$R/recommendation_gans_amd/_variants/librg_hip_${name%%+*}.so;; esac
  [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
  BARGS=""; for kv in $envs; do case $kv in BARGS=*) BARGS=${kv#BARGS=}; BARGS=${BARGS//=/ };; esac; done
  env $envs RG_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline $BARGS > gpurun_out/attr_${TAG}_$name.json 2>gpurun_out/attr_${TAG}_$name.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/attr_${TAG}_$name.json'));print('$spec', 'bench20', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step dense-events', round(d['roofline']['avg_launch_us'],2))" | tee -a $OUT
  (cd /tmp && env $envs RG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/attr_prof_${TAG}_$name -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline $BARGS > $R/gpurun_out/attr_prof_${TAG}_$name.json 2>$R/gpurun_out/attr_prof_${TAG}_$name.err) || exit $?
  python3 - "$R/gpurun_out/attr_prof_${TAG}_$name" "$spec" <<'PY' | tee -a $OUT
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if any(k in n for k in ("mf_pairs", "mf_back", "mf_prepare", "mt_generate", "pipe2", "mf_dense")):
            print(sys.argv[2], n.split("(")[0].split("::")[-1][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
