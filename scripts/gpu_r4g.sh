# round 4: the product dense kernels on micro-style allocations beside the micro stream (one
# process); NCF / NeuMF full-size elementwise parity with the two-order band
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/bin/product_dense > gpurun_out/product_dense_r4g.txt 2>&1 || { cat gpurun_out/product_dense_r4g.txt; exit 1; }
cat gpurun_out/product_dense_r4g.txt
rm -f gpurun_out/parity_elementwise.jsonl
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_configs_gpu.py -k "ncf_full or neumf_full" > gpurun_out/r4g_configs.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r4g_configs.log | tail -5; python3 -c "
import json
for l in open('gpurun_out/parity_elementwise.jsonl'):
    d=json.loads(l)
    if d['n_fail'] or d['n_out']: print(d['tag'], d['n_out'], d['n_fail'], '%.2e' % d['max_rel'])
"; exit $rc
