# GPU box: kernel traces + HBM PMC (FETCH_SIZE / WRITE_SIZE, one per pass) of lazy-pass variants vs eager.
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/lzprof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in "RG_LAZY_SPEC=1 RG_LAZY_DBG=1" "RG_LAZY_SPEC=0 RG_LAZY_DBG=1" "RG_LAZY=0"; do
  tag=$(echo "$v" | tr ' =' '__')
  export $v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b_$tag.json 2>$OUT/b_$tag.err || exit $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/pmc_${tag}_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2>$OUT/pmc_${tag}_$C.err || exit $?
  done
  unset RG_LAZY_SPEC RG_LAZY_DBG RG_LAZY
  echo "$v done"
done
