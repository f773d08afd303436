# GPU box: the pipelined MF step -- bit-identity tests, then the bench A/B against the split step
# (RG_PIPE=0 / 1, cold-row workgroup counts) and a kernel-stats profile.  Usage: bash scripts/gpu_pipe.sh
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_pipe_gpu.py > gpurun_out/r4j_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4j_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "split|RG_PIPE=0" "pipe|RG_PIPE=1" "pipe_c1k|RG_PIPE=1 RG_PIPE_COLD1=1024" "pipe_c4k|RG_PIPE=1 RG_PIPE_COLD1=4096"; do
  IFS='|' read name envs <<< "$cfg"
  for st in "20 5" "200 20"; do
    set -- $st
    env $envs timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/r4j.json 2>gpurun_out/r4j.err || { tail -5 gpurun_out/r4j.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4j.json')); r=d['roofline']; print('$name', $1, round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step; kernel', round(r['avg_launch_us'],1), 'us', d.get('final_loss'))" | tee -a gpurun_out/r4j_ab.txt
  done
done
(cd /tmp && RG_PIPE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4j_prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r4j_prof.json 2>$R/gpurun_out/r4j_prof.err) || exit $?
python3 - "$R/gpurun_out/r4j_prof" <<'PY' | tee -a gpurun_out/r4j_ab.txt
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mf_" in r["Name"]:
            print(r["Name"].split("(")[0][-70:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
