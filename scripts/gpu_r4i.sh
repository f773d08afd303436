# round 4: how much of the pair pass hides beside the dense pass (two streams, timing only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/overlap_probe.py > gpurun_out/overlap_r4i.txt 2>gpurun_out/overlap_r4i.err || { tail -20 gpurun_out/overlap_r4i.err; exit 1; }
cat gpurun_out/overlap_r4i.txt
