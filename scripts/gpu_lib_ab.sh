# GPU box: same-box A/B of library variants (python -m recommendation_gans_amd.build --variant NAME -D...).
# For each NAME (base = the product library): the MF / plan parity tests against that library,
# the bench at 20/5 and 200/20, and a kernel-trace profile (per-kernel average durations).
# Usage: bash scripts/gpu_lib_ab.sh TAG base pb512 ...     (tests skipped if NOTEST=1)
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for name in "$@"; do
  if [ "$name" = base ]; then lib=$R/recommendation_gans_amd/librg_hip.so
  else lib=$R/recommendation_gans_amd/_variants/librg_hip_$name.so; fi
  [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
  if [ "${NOTEST:-0}" != 1 ]; then
    RG_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      -m gpu tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_plan_gpu.py > gpurun_out/lab_tests_${TAG}_$name.log 2>&1
    rc=$?; echo "$name tests exit=$rc"; tail -2 gpurun_out/lab_tests_${TAG}_$name.log
    [ $rc -eq 0 ] || exit $rc
  fi
  for st in "20 5" "200 20"; do
    set -- $st
    RG_LIB=$lib timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/lab_${TAG}_${name}_$1.json 2>gpurun_out/lab_${TAG}_${name}_$1.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/lab_${TAG}_${name}_$1.json'));print('$name', $1, round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), repr(d.get('final_loss')))"
  done
  (cd /tmp && RG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lab_prof_${TAG}_$name -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/lab_prof_${TAG}_$name.json 2>$R/gpurun_out/lab_prof_${TAG}_$name.err) || exit $?
  python3 - "$R/gpurun_out/lab_prof_${TAG}_$name" "$name" <<'EOF'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mf_pairs" in r["Name"] or "mf_back" in r["Name"] or "mf_prepare" in r["Name"]:
            print(sys.argv[2], r["Name"].split("(")[0][-60:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
EOF
done
