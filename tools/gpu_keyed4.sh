#!/bin/bash
# Four-side keyed latency kernel: GPU parity tests, cached-key latency, kernel
# durations (rocprofv3 --kernel-trace --stats) at 1 and 1000 signatures per call.
#   bash tools/gpu_keyed4.sh OUT
set -eu
out=$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_keycache.py tests/test_gpu_verify.py tests/test_gpu_multidev.py > "$out/tests.log" 2>&1
PV_LAT_CACHED=1 PV_LAT_SIZES=1,16,100,1000 timeout -k 10 200 python3 tools/latency.py > "$out/lat.log" 2>&1
for n in 1 1000; do
  PV_LAT_CACHED=1 PV_LAT_SIZES=$n timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof_$n" -o run -- python3 tools/latency.py > "$out/prof_$n.log" 2>&1
done
echo done
