#!/bin/bash
# round 3 batch G: last host chunk on the device schedule (A/B vs all fused).
set -u
out=${1:-gpurun_out/r03_g}
mkdir -p "$out"
echo "[g] $(date +%T) tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_multidev.py tests/test_gpu_keycache.py -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 ; rc=$?; tail -3 "$out/tests.log"; [ $rc -eq 0 ] && \
echo "[g] $(date +%T) ab" && timeout -k 10 300 python tools/ab_host_fused.py 10 > "$out/ab.jsonl" 2> "$out/ab.err" && cat "$out/ab.jsonl" && \
echo "[g] $(date +%T) trace" && PV_HOST_TRACE=1 timeout -k 10 120 python tools/ab_host_fused.py 1 > /dev/null 2> "$out/trace.err" && echo "[g] done"
