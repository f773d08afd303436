# GPU box: the wave-specialised optimizer GEMM (A/B build, RG_GEMM_WS=1) against the product's
# epilogue form: the GEMM tests (both forms, bit-identity) and the cGAN step tests under the
# wave-specialised form, the isolated W1S / WH updates, the cGAN bench line and a kernel-trace
# profile per form.  Build the A/B library first (build.py --variant ab -DRG_AB=1).
# Usage: bash scripts/gpu_gan_ws.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
AB=$R/recommendation_gans_amd/_variants/librg_hip_ab.so
lib() { if [ "$1" = 1 ]; then echo $AB; else echo $R/recommendation_gans_amd/librg_hip.so; fi; }
RG_LIB=$AB RG_GEMM_WS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gan_gpu.py > gpurun_out/gan_ws_tests_$TAG.log 2>&1
rc=$?; echo "gan tests (ws default 1) exit=$rc"; tail -2 gpurun_out/gan_ws_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
RG_LIB=$AB timeout -k 10 300 python3 scripts/gemm_bench.py --rms-only --ws-ab > gpurun_out/gan_ws_gemm_$TAG.jsonl 2>&1 || { tail -5 gpurun_out/gan_ws_gemm_$TAG.jsonl; exit 1; }
cat gpurun_out/gan_ws_gemm_$TAG.jsonl
for rep in 1 2; do for m in 0 1; do
  RG_LIB=$(lib $m) RG_GEMM_WS=$m timeout -k 10 300 python3 bench.py --model gan --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/gan_ws_bench_${TAG}_${m}_$rep.json 2>gpurun_out/gan_ws_bench_${TAG}_${m}_$rep.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/gan_ws_bench_${TAG}_${m}_$rep.json'));print('ws $m rep $rep', round(d['value']), d['unit'], round(d['ms_per_step'],4), 'ms/step', d['roofline']['frac'])"
done; done
for m in 0 1; do
  (cd /tmp && RG_LIB=$(lib $m) RG_GEMM_WS=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gan_ws_prof_${TAG}_$m -o run -- python3 $R/bench.py --model gan --steps 25 --warmup 5 --no-cpu-baseline > $R/gpurun_out/gan_ws_prof_${TAG}_$m.json 2>$R/gpurun_out/gan_ws_prof_${TAG}_$m.err) || exit $?
  python3 - "$R/gpurun_out/gan_ws_prof_${TAG}_$m" "$m" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:6]:
        print("ws", sys.argv[2], r["Name"].split("(")[0][-70:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total")
PY
done
