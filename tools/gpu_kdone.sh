#!/bin/bash
# In-kernel completion word for all-cached zero-copy calls (default build) vs
# the k_signal launch behind the kernel (lib/ab/signal_launch.so, previous
# commit; both builds share the current Python wrapper): the -m gpu suite, then
# interleaved host-call latencies, cached and uncached keys.
#   bash tools/gpu_kdone.sh OUT
set -u
out=${1:-gpurun_out/kdone}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_suite.sh "$out/suite" && \
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/signal_launch.so; do
    tag=$(basename $lib .so)
    for c in 1 0; do
      PLENUM_GPU_LIB=$lib PV_LAT_CACHED=$c PV_LAT_SIZES=1,16,100,1000 timeout -k 10 200 python3 tools/latency.py 2>/dev/null | sed "s/^{/{\"lib\": \"$tag\", \"rep\": $r, /" >> "$out/lat_ab.jsonl" || exit 1
    done
  done
done && echo done
