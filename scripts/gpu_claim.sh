# GPU box: claimed list slots -- parity tests, then same-box A/B of the MF bench (RG_MF_CLAIM 0/1)
# and a rocprof kernel-stats pass of the claimed step.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_claim_gpu.py tests/test_mf_gpu.py tests/test_dropin_gpu.py tests/test_lazy_gpu.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for c in 0 1; do
    RG_MF_CLAIM=$c timeout -k 10 180 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/claim_${TAG}_c${c}_$k.json 2>gpurun_out/claim_${TAG}_c${c}_$k.err || exit $?
    python - gpurun_out/claim_${TAG}_c${c}_$k.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], round(d["value"] / 1e6, 2), "M/s", round(d["ms_per_step"] * 1e3, 2), "us/step")
PY
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/claimprof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/claimprof_$TAG.json 2>$GRAFT_REPO_ROOT/gpurun_out/claimprof_$TAG.err && echo prof-ok
