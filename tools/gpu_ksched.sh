#!/bin/bash
# Keyed latency kernel with the hash wave's per-block schedule lanes (default
# build) vs inline schedules (lib/ab/sched_inline.so, previous commit): the -m gpu
# suite, kernel durations at n = 1, interleaved host-call latencies.
#   bash tools/gpu_ksched.sh OUT
set -u
out=${1:-gpurun_out/ksched}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_suite.sh "$out/suite" && \
for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/sched_inline.so; do
  tag=$(basename $lib .so)
  PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof_$tag" -o run -- python3 tools/latency.py > "$out/prof_$tag.log" 2>&1 || exit 1
done && \
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/sched_inline.so; do
    tag=$(basename $lib .so)
    PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1,16,100,1000,4096 timeout -k 10 200 python3 tools/latency.py 2>/dev/null | sed "s/^{/{\"lib\": \"$tag\", \"rep\": $r, /" >> "$out/lat_ab.jsonl" || exit 1
  done
done && echo done
