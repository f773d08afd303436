# cGAN GEMM knob A/B: per setting "ONESTAGE:OPTSTAGES:PARTTARGET", a bench line (+ gemm_bench.py with GEMMS=1)
set -o pipefail
mkdir -p gpurun_out
for KV in ${SETTINGS:-0:2:512 1:7:768}; do
  IFS=: read -r RG_GEMM_1STAGE RG_GEMM_OPT_STAGES RG_GAN_PART_TARGET <<< "$KV"
  export RG_GEMM_1STAGE RG_GEMM_OPT_STAGES RG_GAN_PART_TARGET
  if [ -n "$GEMMS" ]; then timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_ab_$KV.jsonl 2>&1 || exit 1; fi
  timeout -k 10 300 python bench.py --model gan --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/gan_ab_$KV.json 2> gpurun_out/gan_ab_$KV.err || exit 1
  echo "== $KV"
  python -c "import json;d=json.load(open('gpurun_out/gan_ab_$KV.json'));print('gan', round(d['value']), d['ms_per_step'], d['roofline']['frac'])"
done
