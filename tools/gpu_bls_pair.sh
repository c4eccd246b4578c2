#!/bin/bash
# Lane-pair BLS check kernel on the GPU: the BLS GPU tests on the shipped
# library (k_bls_verify_pair), then the c3bls bench on it and on the one-lane
# variant (-D PV_BLS_ONE_LANE, lib/ab/one_lane.so), then the one-check latency.
#   bash tools/gpu_bls_pair.sh OUT
set -u
out=${1:-gpurun_out/bls_pair}
mkdir -p "$out"
echo "[pair] $(date +%T) tests" && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_bls_multi.py -x -v --timeout 300 --timeout-method thread -m gpu > "$out/tests.log" 2>&1 && \
echo "[pair] $(date +%T) bench pair" && \
timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls_pair.json" 2> "$out/c3bls_pair.err" && \
echo "[pair] $(date +%T) bench one-lane" && \
PLENUM_GPU_LIB=indy-plenum_amd/lib/ab/one_lane.so timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls_one.json" 2> "$out/c3bls_one.err" && \
echo "[pair] done"
