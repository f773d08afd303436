# GPU box: same-box A/B of dense-pass variants at d = 128 and d = 64 (variants built with
# build.py --variant NAME --only rg_mf.hip -D...).  Usage: bash scripts/gpu_ab_dense_layouts.sh
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for rep in 1 2; do for v in base v128k4 pg2; do
  if [ $v = base ]; then L=$R/recommendation_gans_amd/librg_hip.so; else L=$R/recommendation_gans_amd/_variants/librg_hip_$v.so; fi
  for dim in 128 64; do
    RG_LIB=$L timeout -k 10 200 python3 bench.py --dim $dim --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab128_${v}_${dim}_$rep.json 2>gpurun_out/ab128_${v}_${dim}_$rep.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/ab128_${v}_${dim}_$rep.json'));print('$v d$dim rep $rep', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2))"
  done
done; done
