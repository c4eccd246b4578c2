#!/bin/bash
# Round-5 closing line on the final build: the -m gpu suite + smoke, the default
# bench line (C2 + other configs + end to end + latency + CPU baseline) and the
# rocprofv3 kernel stats of the C2 bench.
#   bash tools/gpu_closing_r05.sh OUT
set -u
out=${1:-gpurun_out/closing5}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_suite.sh "$out/suite" && \
echo "[closing] $(date +%T) bench" && \
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" && \
echo "[closing] $(date +%T) stats" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_c2" -o run -- python3 bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline --no-e2e --no-other-configs > "$out/prof_c2.log" 2>&1 && echo "[closing] done"
