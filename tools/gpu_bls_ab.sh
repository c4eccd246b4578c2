#!/bin/bash
# BLS engine: full-size c3bls bench at 2 and 1 waves/SIMD (variant library),
# then a rocprofv3 kernel-trace of a smaller run.
#   bash tools/gpu_bls_ab.sh OUT
set -u
out=${1:-gpurun_out/bls_ab}
mkdir -p "$out"
echo "[bls_ab] $(date +%T) w2 full" && timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls_w2.json" 2> "$out/c3bls_w2.err" && \
echo "[bls_ab] $(date +%T) w1 full" && PLENUM_GPU_LIB=indy-plenum_amd/lib/libplenum_verify_blsw1.so timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls_w1.json" 2> "$out/c3bls_w1.err" && \
echo "[bls_ab] $(date +%T) rocprof" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --config c3bls --n 500000 --steps 2 --warmup 1 --no-cpu-baseline > "$out/prof.log" 2>&1 && echo "[bls_ab] done"
