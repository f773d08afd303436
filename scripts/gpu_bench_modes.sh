# GPU box: every bench.py mode once at a few steps (a smoke of the bench's own code paths, not a
# measurement): MF losses and optimizers, d = 32 / 128, no prefetch, the data-parallel code paths
# at N = 1 (owner with and without a one-rank RCCL communicator, global_stream, user_shard), the
# emulated rank, host-ahead, NCF (E = 64 wave kernel, E = 32 tile kernel) / NeuMF, cGAN, eval.
# Usage: bash scripts/gpu_bench_modes.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
OUT=gpurun_out/bench_modes_$TAG.txt
: > $OUT
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i + 1))
  timeout -k 10 240 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline $line > gpurun_out/bm_${TAG}_$i.json 2> gpurun_out/bm_${TAG}_$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAIL rc=$rc: $line" | tee -a $OUT; tail -5 gpurun_out/bm_${TAG}_$i.err | tee -a $OUT; exit $rc; fi
  python3 -c "import json;d=json.loads(open('gpurun_out/bm_${TAG}_$i.json').read().strip().splitlines()[-1]);print('ok', repr('$line'), round(d['value'], 1), d['unit'], d.get('final_loss'))" | tee -a $OUT
done <<'EOF'
--loss pointwise
--loss hinge
--loss adaptive_hinge
--optim sgd
--optim rms
--dim 32
--dim 128
--no-prefetch
--dp owner --dp-at-1
--dp owner --dp-at-1 --comm-at-1
--dp global_stream --dp-at-1
--dp user_shard --dp-at-1
--emulate-rank 3/8
--host-ahead 0.5
--model ncf
--model ncf --dim 32
--model neumf
--model gan
--model eval
EOF
echo "all modes ok" | tee -a $OUT
