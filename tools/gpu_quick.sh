#!/bin/bash
# GPU test suite + C2/C3/C4 bench lines (no profiling).  Run on the GPU box:
#   bash tools/gpu_quick.sh gpurun_out/quick
set -u
out=${1:-gpurun_out/quick}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1 && \
timeout -k 10 240 python bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err" && \
timeout -k 10 240 python bench.py --config c3 > "$out/bench_c3.json" 2> "$out/bench_c3.err" && \
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 > "$out/bench_c4.json" 2> "$out/bench_c4.err"
echo "rc=$?"
