# round 4: is the dense pass bound by the MT walk it hosts (inline generation)?  A/B of the
# word source (inline walk in the dense pass vs 8 / 16-unit slots on the generator stream),
# product and lean libraries; then the micro floor with real data / pollution; then parity.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for lib in base lean; do
  if [ $lib = base ]; then L=$R/recommendation_gans_amd/librg_hip.so; else L=$R/recommendation_gans_amd/_variants/librg_hip_$lib.so; fi
  for envs in "RG_MT_INLINE=1" "RG_MT_INLINE=0" "RG_MT_INLINE=0 RG_MT_UNITS=16" "RG_MT_INLINE=0 RG_MT_JUMP=1"; do
    for st in "20 5" "200 20"; do
      set -- $st
      env RG_LIB=$L $envs timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/r4f.json 2>gpurun_out/r4f.err || exit $?
      python -c "import json; d=json.load(open('gpurun_out/r4f.json')); r=d['roofline']; print('$lib', '$envs', $1, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; dense', round(r['avg_launch_us'],1), 'us', d.get('final_loss'))"
    done
  done
done
(cd /tmp && RG_MT_INLINE=0 RG_LIB=$R/recommendation_gans_amd/_variants/librg_hip_lean.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4f_prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r4f_prof.json 2>$R/gpurun_out/r4f_prof.err) || exit $?
python3 - "$R/gpurun_out/r4f_prof" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"].split("(")[0][-70:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
timeout -k 10 120 ./scripts/micro/bin/dense_floor 1 > gpurun_out/dense_floor_r4f.txt 2>&1 || exit $?
cat gpurun_out/dense_floor_r4f.txt
rm -f gpurun_out/parity_elementwise.jsonl
timeout -k 10 1000 python -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_configs_gpu.py tests/test_ncf_gpu.py -k "full_size or owner or rejects" > gpurun_out/r4f_configs.log 2>&1
rc=$?; grep -E "ParityReport|passed|failed" gpurun_out/r4f_configs.log | tail -80; exit $rc
