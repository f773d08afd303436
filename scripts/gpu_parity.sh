# GPU box: the full-size configuration tests with elementwise parity reports (C2, C3, C5 owner,
# NeuMF; tests/parity_report.py) -> gpurun_out/parity_elementwise.jsonl, then a summary of the
# elements outside the band.  Usage: bash scripts/gpu_parity.sh TAG [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
K=${2:-"mf_full_size or owner or ncf_full or neumf_full"}
rm -f gpurun_out/parity_elementwise.jsonl
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_configs_gpu.py -k "$K" > gpurun_out/parity_$TAG.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/parity_$TAG.log | tail -30
python3 - <<'PY'
import json, os
p = "gpurun_out/parity_elementwise.jsonl"
if os.path.exists(p):
    for l in open(p):
        d = json.loads(l)
        print(f"{d['tag']:40s} n={d['n']:>10d} out_1e-5={d['n_out']:>7d} ({d['frac_out']:.2e}) "
              f"fail={d['n_fail']} max_rel={d['max_rel']:.2e}")
PY
exit $rc
