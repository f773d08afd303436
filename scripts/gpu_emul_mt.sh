# GPU box: rank 0 of 8 emulated (bench.py --emulate-rank 0/8) with 8 / 16 / 32 steps per MT ring
# slot (RG_MT_UNITS): the jump-ahead walk's fixed per-slot cost spread over more steps.
set -o pipefail
mkdir -p gpurun_out
for g in 8 16 32 8; do
  RG_MT_UNITS=$g timeout -k 10 300 python3 bench.py --gpus 1 --steps 64 --warmup 16 --no-cpu-baseline --emulate-rank 0/8 > gpurun_out/emul_mt$g.json 2>gpurun_out/emul_mt$g.err || { tail -3 gpurun_out/emul_mt$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/emul_mt$g.json'));print('units $g', round(d['ms_per_step']*1e3,2), 'us/step', round(d['user_update_us'],1), round(d['value']/1e6,1), 'M/s projected')"
done
