# GPU box: decomposition of the overlapped MF step (scripts/mf_step_probe.py), one rocprof pass per variant
set -o pipefail
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in split fused_scan fused_owner front_pairs_only two_stream serial; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/probe/$v -o run -- python $R/scripts/mf_step_probe.py --variant $v --iters 40 > $R/gpurun_out/probe/$v.txt 2>&1) || exit $?
  grep -v amdgpu.ids gpurun_out/probe/$v.txt | head -2
  python - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/probe/{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "rg::" in n and "mt_" not in n:
        print(f'   {r["Calls"]:>4} {float(r["AverageNs"])/1000:7.1f}us {n.split("(")[0][:60]}')
PY
done
for cfg in "RG_MT_JUMP=0" "RG_MT_JUMP=1" "RG_FUSED=0 RG_MT_JUMP=0" "RG_FUSED=0 RG_MT_JUMP=0 RG_MT_UNITS=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b.json 2>/dev/null || exit $?
  echo "$cfg" $(python -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1), round(d['host_enqueue_us_per_step'],1))")
done
