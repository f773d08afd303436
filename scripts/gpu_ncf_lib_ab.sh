# GPU box: same-box A/B of NCF library variants (python -m recommendation_gans_amd.build --variant NAME
# --only rg_ncf.hip ...).  The NCF / NeuMF GPU tests against every non-base variant first, then per
# variant, interleaved twice: the NCF bench line and a rocprofv3 kernel-trace of it (average
# ncf_wave_kernel and tail-launch durations).
# Usage: [NCFMODEL=neumf] bash scripts/gpu_ncf_lib_ab.sh TAG base NAME ...
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=gpurun_out/ncf_ab_$TAG.txt
libof() { if [ "$1" = base ]; then echo $R/recommendation_gans_amd/librg_hip.so; else echo $R/recommendation_gans_amd/_variants/librg_hip_$1.so; fi; }
for name in "$@"; do
  lib=$(libof $name); [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
  [ "$name" = base ] && continue
  RG_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -m gpu tests/test_ncf_wave_gpu.py tests/test_ncf_gpu.py tests/test_neumf_gpu.py tests/test_mf_gpu.py > gpurun_out/ncf_ab_tests_${TAG}_$name.log 2>&1
  rc=$?; echo "$name tests exit=$rc" | tee -a $OUT; tail -2 gpurun_out/ncf_ab_tests_${TAG}_$name.log
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for name in "$@"; do
    lib=$(libof $name)
    RG_LIB=$lib timeout -k 10 200 python3 bench.py --model ${NCFMODEL:-ncf} --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ncf_ab_${TAG}_$name.json 2>gpurun_out/ncf_ab_${TAG}_$name.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/ncf_ab_${TAG}_$name.json'));print('$name', 'bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step')" | tee -a $OUT
    (cd /tmp && RG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ncf_ab_prof_${TAG}_${name}_$rep -o run -- python3 $R/bench.py --model ${NCFMODEL:-ncf} --steps 40 --warmup 5 --no-cpu-baseline > /dev/null 2>$R/gpurun_out/ncf_ab_prof_${TAG}_$name.err) || exit $?
    python3 - "$R/gpurun_out/ncf_ab_prof_${TAG}_${name}_$rep" "$name" <<'EOF' | tee -a $OUT
import csv, glob, sys
out = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "ncf_wave_kernel" in n or "mf_back_kernel" in n:
            out.append(f"{n.split('(')[0][-34:]} {r['Calls']} x {float(r['AverageNs']) / 1e3:.2f} us")
print(sys.argv[2], "; ".join(out))
EOF
  done
done
