#!/bin/bash
# round 3 batch F: keyed latency kernel with S B before the barrier; C4 (k_keys) and C2 benches.
#   bash tools/gpu_r03_f.sh OUT
set -u
out=${1:-gpurun_out/r03_f}
mkdir -p "$out"
S=1,16,100,1000,2048,4096,8192
echo "[f] $(date +%T) tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_verify.py tests/test_gpu_device.py -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 ; rc=$?; tail -3 "$out/tests.log"; [ $rc -eq 0 ] && \
echo "[f] $(date +%T) latency" && \
for c in 0 1; do PV_LAT_CACHED=$c PV_LAT_SIZES=$S timeout -k 10 300 python tools/latency.py 2>/dev/null >> "$out/lat.jsonl" || exit 1; done && cat "$out/lat.jsonl" && \
echo "[f] $(date +%T) c4" && timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$out/c4.json" 2> "$out/c4.err" && \
echo "[f] $(date +%T) c2" && timeout -k 10 300 python bench.py --no-cpu-baseline > "$out/c2.json" 2> "$out/c2.err" && tail -c 600 "$out/c2.json" && echo "[f] done"
