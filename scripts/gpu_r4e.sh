# round 4: micro floor with real data / Infinity-Cache pollution; full-size parity with elementwise reports
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/micro/bin/dense_floor 1 > gpurun_out/dense_floor_r4e.txt 2>&1 || exit $?
cat gpurun_out/dense_floor_r4e.txt
rm -f gpurun_out/parity_elementwise.jsonl
timeout -k 10 1000 python -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_configs_gpu.py tests/test_ncf_gpu.py -k "full_size or owner or rejects" > gpurun_out/r4e_configs.log 2>&1
rc=$?; grep -E "ParityReport|passed|failed" gpurun_out/r4e_configs.log | tail -80; exit $rc
