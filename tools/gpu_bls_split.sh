#!/bin/bash
# Where k_bls_verify's time goes: the c3bls bench on the shipped library and on
# a variant without the final exponentiation (-D PV_BLS_AB_MILLER_ONLY, verdicts
# meaningless), each under a rocprofv3 kernel trace.
#   bash tools/gpu_bls_split.sh OUT
set -u
out=${1:-gpurun_out/bls_split}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
echo "[split] $(date +%T) full" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/full" -o run -- python3 bench.py --config c3bls --n 500000 --steps 2 --warmup 1 --no-cpu-baseline > "$out/full.json" 2> "$out/full.err" && \
echo "[split] $(date +%T) miller only" && \
PLENUM_GPU_LIB=indy-plenum_amd/lib/ab/miller_only.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/miller" -o run -- python3 bench.py --config c3bls --n 500000 --steps 2 --warmup 1 --no-cpu-baseline > "$out/miller.json" 2> "$out/miller.err" && \
echo "[split] done"
