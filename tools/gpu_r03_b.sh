#!/bin/bash
# round 3 batch B: BLS tests + bench with the inlined Miller / cyclotomic loops,
# C4 bench with 128-byte-aligned key tables, then k_keys PMC passes.
#   bash tools/gpu_r03_b.sh OUT
set -u
out=${1:-gpurun_out/r03_b}
mkdir -p "$out"
echo "[b] $(date +%T) bls tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 && tail -1 "$out/tests.log" && \
echo "[b] $(date +%T) c3bls" && timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 > "$out/c3bls.json" 2> "$out/c3bls.err" && \
echo "[b] $(date +%T) c4" && timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$out/c4.json" 2> "$out/c4.err" && \
echo "[b] $(date +%T) pmc keys" && bash tools/pmc_keys.sh "$out/pmc_keys" 2000000 && echo "[b] done"
