# GPU box: the NCF / NeuMF step's GPU-side time (bench.py --host-ahead) against the wall time, and a
# kernel trace of each for the gaps between the step's launches.  Usage: bash scripts/gpu_ncf_gaps.sh TAG
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in ncf neumf; do
  timeout -k 10 300 python3 bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/gaps_${m}_$TAG.json 2> gpurun_out/gaps_${m}_$TAG.err || exit 1
  timeout -k 10 300 python3 bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline --host-ahead 30 > gpurun_out/gaps_${m}_ahead_$TAG.json 2> gpurun_out/gaps_${m}_ahead_$TAG.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/gaps_${m}_$TAG.json')); a=json.load(open('gpurun_out/gaps_${m}_ahead_$TAG.json')); print('$m wall', round(d['ms_per_step']*1e3,1), 'us/step host', round(d['host_enqueue_us_per_step'],1), '| ahead', round(a['gpu_ahead_us_per_step'],1))"
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gaps_prof_${m}_$TAG -o run -- python3 $R/bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > /dev/null 2>$R/gpurun_out/gaps_prof_${m}_$TAG.err) || exit 1
done
echo done
