# GPU box: the NCF wave kernel's forward one example block at a time (RG_NCF_FWD_BLOCKWISE) at 32-
# and 48-row tiles, against the product: the wave-kernel tests on each variant, then an NCF bench
# line and the kernel's rocprof average per library.  Usage: bash scripts/gpu_ncf_fwd.sh TAG variant...
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/recommendation_gans_amd/librg_hip.so
  [ $v = base ] || lib=$R/recommendation_gans_amd/_variants/librg_hip_$v.so
  RG_LIB=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_ncf_wave_gpu.py > gpurun_out/ncffwd_tests_${v}_$TAG.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/ncffwd_tests_${v}_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
  RG_LIB=$lib timeout -k 10 300 python3 bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ncffwd_${v}_$TAG.json 2>gpurun_out/ncffwd_${v}_$TAG.err || exit 1
  (cd /tmp && RG_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ncffwd_prof_${v}_$TAG -o run -- python3 $R/bench.py --model ncf --steps 30 --warmup 5 --no-cpu-baseline > /dev/null 2>$R/gpurun_out/ncffwd_prof_${v}_$TAG.err) || exit 1
  python3 - "$R/gpurun_out/ncffwd_prof_${v}_$TAG" "$v" "gpurun_out/ncffwd_${v}_$TAG.json" <<'PY'
import csv, glob, json, sys
d = json.load(open(sys.argv[3]))
k = [r for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(f))
     if "ncf_wave_kernel" in r["Name"] or "mf_back_kernel" in r["Name"]]
print(sys.argv[2], "NCF", round(d["value"] / 1e6, 2), "M/s", round(d["ms_per_step"] * 1e3, 1), "us/step;",
      "; ".join(f"{r['Name'].split('(')[0][-40:]} {round(float(r['AverageNs']) / 1e3, 2)} us" for r in k))
PY
done
