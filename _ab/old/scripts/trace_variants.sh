# kernel traces of bench variants.  Usage: bash scripts/trace_variants.sh TAG "name:ENV=val:args" ...
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
  cd /tmp
  [ -n "$envs" ] && export $envs
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_${TAG}_$name -o run -- python $R/bench.py --steps 60 --warmup 10 --no-cpu-baseline $args > $R/gpurun_out/tr_${TAG}_$name.json 2>/dev/null || exit $?
  timeout -k 10 300 python $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline $args > $R/gpurun_out/b_${TAG}_$name.json 2>/dev/null || exit $?
  cd $R && python scripts/trace_summary.py gpurun_out/tr_${TAG}_$name && python -c "import json; d=json.load(open('gpurun_out/b_${TAG}_$name.json')); print('  bench', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step')"
done
