# GPU box (timing only): the pipelined step with its pair workgroups idle (x1: wait, no pair
# pass; x3: not even the wait) against the full pipelined step and the split step.
set -o pipefail
mkdir -p gpurun_out
for cfg in "split|RG_PIPE=0|" "pipe|RG_PIPE=1|" "pipe_x1|RG_PIPE=1|recommendation_gans_amd/_variants/librg_hip_pipex1.so" "pipe_x3|RG_PIPE=1|recommendation_gans_amd/_variants/librg_hip_pipex3.so"; do
  IFS='|' read name envs lib <<< "$cfg"
  env $envs ${lib:+RG_LIB=$lib} timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/px.json 2>gpurun_out/px.err
  python -c "import json; d=json.load(open('gpurun_out/px.json')); r=d['roofline']; print('$name', round(d['ms_per_step']*1e3,1), 'us/step; kernel', round(r['avg_launch_us'],1), 'us')" || tail -3 gpurun_out/px.err
done
