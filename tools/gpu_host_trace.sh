#!/bin/bash
# Host-side timings of the 1M host-buffer call (PV_HOST_TRACE=1: per-chunk slot /
# gather / enqueue times on stderr) for a few gather-thread counts.
#   bash tools/gpu_host_trace.sh OUT
set -u
out=${1:-gpurun_out/htrace}
mkdir -p "$out"
for t in 8 16 4; do
  PV_HOST_TRACE=1 PV_HOST_COPY_THREADS=$t timeout -k 10 240 python3 tools/e2e_trace.py > "$out/t$t.log" 2>&1 || exit 1
done
echo done
