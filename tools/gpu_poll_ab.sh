#!/bin/bash
# Interleaved host-call latencies: polled completion (default build) vs stream
# synchronize (lib/ab/zc_sync.so, -D PV_ZC_POLL=0), cached and uncached keys.
#   bash tools/gpu_poll_ab.sh OUT
set -u
out=${1:-gpurun_out/pollab}
mkdir -p "$out"
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/zc_sync.so; do
    tag=$(basename $lib .so)
    for c in 1 0; do
      PLENUM_GPU_LIB=$lib PV_LAT_CACHED=$c PV_LAT_SIZES=1,16,100,1000 timeout -k 10 200 python3 tools/latency.py 2>/dev/null | sed "s/^{/{\"lib\": \"$tag\", \"rep\": $r, /" >> "$out/lat_ab.jsonl" || exit 1
    done
  done
done && echo done
