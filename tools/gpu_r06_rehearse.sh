#!/bin/bash
# Round 6: the self-launching bench at N > 1 rehearsed on a one-GPU box (gloo,
# every rank on GPU 0), C2 at 4 ranks and C4 at 2, and the C3 line with the wide
# key preparation timed in its stages.
#   bash tools/gpu_r06_rehearse.sh OUT
set -u
out=${1:-gpurun_out/r06reh}
mkdir -p "$out"
echo "[reh] $(date +%T) c2 x4" && \
PV_BENCH_BACKEND=gloo PV_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 4 --steps 5 --warmup 2 \
    --no-e2e > "$out/c2_n4.json" 2> "$out/c2_n4.err" && \
echo "[reh] $(date +%T) c4 x2" && \
PV_BENCH_BACKEND=gloo PV_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --config c4 --steps 3 \
    --warmup 1 --n 2000000 --no-cpu-baseline > "$out/c4_n2.json" 2> "$out/c4_n2.err" && \
echo "[reh] $(date +%T) c3" && \
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c3.json" 2> "$out/c3.err" && \
echo "[reh] done"
