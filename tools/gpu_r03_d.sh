#!/bin/bash
# round 3 batch D: keyed latency kernel + persistent key cache.  Key-cache and
# verify parity tests, host-call latency with and without cached keys.
#   bash tools/gpu_r03_d.sh OUT
set -u
out=${1:-gpurun_out/r03_d}
mkdir -p "$out"
echo "[d] $(date +%T) tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_verify.py tests/test_gpu_plenum.py -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 ; rc=$?; tail -3 "$out/tests.log"; [ $rc -eq 0 ] && \
echo "[d] $(date +%T) latency" && PV_LAT_SIZES=1,16,100,1000,4096,8192,16384,32768 timeout -k 10 300 python tools/latency.py > "$out/lat_uncached.jsonl" 2>&1 && \
PV_LAT_CACHED=1 PV_LAT_SIZES=1,16,100,1000,4096,8192,16384,32768 timeout -k 10 300 python tools/latency.py > "$out/lat_cached.jsonl" 2>&1 && \
cat "$out/lat_uncached.jsonl" "$out/lat_cached.jsonl" && \
echo "[d] $(date +%T) rocprof latency" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
PV_LAT_CACHED=1 PV_LAT_SIZES=1,100,1000 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_lat_cached" -o run -- python3 tools/latency.py > "$out/prof_lat_cached.log" 2>&1 && echo "[d] done"
