#!/bin/bash
# Round-5 closing evidence on the final build: the default bench line (C2 + the
# other configs + end-to-end + small-call latency + CPU baseline), rocprofv3
# kernel stats of the C2 bench (pipelined and --sequential), and the C2 curve
# kernel's PMC passes (roofline.traffic).
#   bash tools/gpu_final_r05.sh OUT
set -u
out=${1:-gpurun_out/final5}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[final] $(date +%T) bench" && \
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" && \
echo "[final] $(date +%T) stats" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_c2" -o run -- python3 bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline --no-e2e --no-other-configs > "$out/prof_c2.log" 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_c2_seq" -o run -- python3 bench.py --steps 10 --warmup 3 \
    --sequential --no-cpu-baseline --no-e2e --no-other-configs > "$out/prof_c2_seq.log" 2>&1 && \
echo "[final] $(date +%T) pmc" && \
bash tools/pmc_passes.sh "$out/pmc_c2" 1000000 && echo "[final] done"
