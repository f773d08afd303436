# GPU box: bench at the driver's 20/5 and at 200/20 under MT generator variants + jump-path kernel trace.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  for st in "20 5" "200 20"; do
    set -- $st
    env $ENVV timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/mtv_${TAG}_${name}_$1.json 2>/dev/null || return $?
    python3 -c "import json;d=json.load(open('gpurun_out/mtv_${TAG}_${name}_$1.json'));print('$name', $1, round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2))"
  done
}
ENVV="RG_MT_JUMP=0" run plain || exit $?
ENVV="RG_MT_JUMP=1" run jump || exit $?
ENVV="RG_MT_JUMP=0 RG_MT_UNITS=2" run plain_g2 || exit $?
ENVV="RG_MT_JUMP=1 RG_MT_UNITS=2" run jump_g2 || exit $?
cd /tmp && RG_MT_JUMP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_jump_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-cpu-baseline > /dev/null 2>&1 && echo prof-ok
