#!/bin/bash
# Keyed latency kernel with LDS-flag hand-offs (default build) vs the block
# barriers (lib/ab/keyed_barrier.so): the -m gpu suite, interleaved host-call
# latencies, kernel durations at n = 1.
#   bash tools/gpu_keyed_flags.sh OUT
set -u
out=${1:-gpurun_out/kflags}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_suite.sh "$out/suite" && \
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/keyed_barrier.so; do
    tag=$(basename $lib .so)
    PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1,16,100,1000,4096 timeout -k 10 200 python3 tools/latency.py 2>/dev/null | sed "s/^{/{\"lib\": \"$tag\", \"rep\": $r, /" >> "$out/lat_ab.jsonl" || exit 1
  done
done && \
for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/keyed_barrier.so; do
  tag=$(basename $lib .so)
  PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof_$tag" -o run -- python3 tools/latency.py > "$out/prof_$tag.log" 2>&1 || exit 1
done && echo done
