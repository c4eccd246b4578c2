#!/bin/bash
# Round-4 BLS evidence on HEAD (lane-pair kernel): the c3bls bench line (with the
# per-call latencies), FETCH / WRITE / SQ passes over it, the kernel-trace stats.
#   bash tools/gpu_bls_pmc_r04b.sh OUT
set -u
out=${1:-gpurun_out/r04bls}
mkdir -p "$out"
echo "[bls] $(date +%T) bench" && \
timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 > "$out/c3bls.json" 2> "$out/c3bls.err" && \
echo "[bls] $(date +%T) pmc" && \
bash tools/pmc_passes.sh "$out/pmc" 500000 --config c3bls && \
echo "[bls] $(date +%T) stats" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --config c3bls \
    --steps 3 --warmup 1 --no-cpu-baseline > "$out/prof.log" 2>&1 && echo "[bls] done"
