#!/bin/bash
# round 3 batch E: zero-copy small host calls (A/B vs copies), cached / uncached keys.
#   bash tools/gpu_r03_e.sh OUT
set -u
out=${1:-gpurun_out/r03_e}
mkdir -p "$out"
S=1,16,100,1000,2048,4096,8192
echo "[e] $(date +%T) tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_verify.py tests/test_gpu_plenum.py tests/test_gpu_c1.py -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 ; rc=$?; tail -3 "$out/tests.log"; [ $rc -eq 0 ] && \
echo "[e] $(date +%T) latency" && \
for zc in 2048 0; do for c in 0 1; do PV_SMALL_ZC_MAX=$zc PV_LAT_CACHED=$c PV_LAT_SIZES=$S timeout -k 10 300 python tools/latency.py 2>/dev/null | sed "s/^{/{\"zc_max\": $zc, /" >> "$out/lat.jsonl" || exit 1; done; done && cat "$out/lat.jsonl" && echo "[e] done"
