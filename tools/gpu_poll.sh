#!/bin/bash
# Host-polled completion of zero-copy calls: the -m gpu suite, then host-call
# latencies (cached and uncached keys) and the keyed kernel's durations.
#   bash tools/gpu_poll.sh OUT
set -u
out=${1:-gpurun_out/poll}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_suite.sh "$out/suite" && \
PV_LAT_CACHED=1 PV_LAT_SIZES=1,16,100,1000,4096 timeout -k 10 200 python3 tools/latency.py > "$out/lat_cached.jsonl" 2>/dev/null && \
PV_LAT_SIZES=1,16,100,1000,4096 timeout -k 10 200 python3 tools/latency.py > "$out/lat_uncached.jsonl" 2>/dev/null && \
PV_LAT_CACHED=1 PV_LAT_SIZES=1,100 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 tools/latency.py > "$out/prof.log" 2>&1 && echo done
