# GPU box: every bench mode once (driver-shaped MF line, d=128 (C5), NCF (C3), NeuMF, cGAN (C4)).
# Usage: bash scripts/gpu_benches.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > gpurun_out/bench_${nm}_$TAG.json 2> gpurun_out/bench_${nm}_$TAG.err || return $?
  python -c "import json;d=json.load(open('gpurun_out/bench_${nm}_$TAG.json'));r=d.get('roofline') or {};c=d.get('cpu_baseline') or {};print('$nm', round(d['value']/1e6,3), round(d['ms_per_step'],4), r.get('frac'), c.get('value'))"
}
run mf --gpus 1 --steps 20 --warmup 5 --cpu-baseline-seconds 10 || exit $?
run mf128 --steps 50 --warmup 5 --dim 128 --no-cpu-baseline || exit $?
run ncf --model ncf --steps 30 --warmup 5 --cpu-baseline-seconds 10 || exit $?
run neumf --model neumf --steps 30 --warmup 5 --no-cpu-baseline || exit $?
run gan --model gan --steps 20 --warmup 3 --no-cpu-baseline || exit $?
run eval --model eval || exit $?
