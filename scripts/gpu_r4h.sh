# round 4: the pipelined dense pass (mf_dense_kernel) vs mf_back_kernel; product harness; parity
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
P=$R/recommendation_gans_amd/_variants/librg_hip_pipe.so
RG_LIB=$P timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_mf_fused_gpu.py tests/test_mf_gpu.py tests/test_plan_gpu.py tests/test_claim_gpu.py > gpurun_out/r4h_tests_pipe.log 2>&1
rc=$?; tail -2 gpurun_out/r4h_tests_pipe.log; [ $rc -eq 0 ] || exit $rc
for cfg in "base|$R/recommendation_gans_amd/librg_hip.so|" "pipe4|$P|RG_DENSE_PER_CU=4" "pipe2|$P|RG_DENSE_PER_CU=2" "pipe8|$P|RG_DENSE_PER_CU=8"; do
  IFS='|' read name L envs <<< "$cfg"
  for st in "20 5" "200 20"; do
    set -- $st
    env RG_LIB=$L $envs timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/r4h.json 2>gpurun_out/r4h.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/r4h.json')); r=d['roofline']; print('$name', $1, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; dense', round(r['avg_launch_us'],1), 'us', d.get('final_loss'))" | tee -a gpurun_out/r4h_ab.txt
  done
done
(cd /tmp && RG_LIB=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4h_prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r4h_prof.json 2>$R/gpurun_out/r4h_prof.err) || exit $?
python3 - "$R/gpurun_out/r4h_prof" <<'PY' | tee -a gpurun_out/r4h_ab.txt
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mf_" in r["Name"]:
            print(r["Name"].split("(")[0][-70:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
timeout -k 10 120 ./scripts/micro/bin/product_dense > gpurun_out/product_dense_r4h.txt 2>&1 || { cat gpurun_out/product_dense_r4h.txt; exit 1; }
cat gpurun_out/product_dense_r4h.txt
