#!/bin/bash
# The flags kernel's paths alone (PV_KEYED_PHASE: 1 no root, 3 hash only, 6 root
# only) and the default build: kernel durations at n = 1, then the -m gpu suite
# and host-call latencies (cached / uncached) of the default build.
#   bash tools/gpu_kflag_phase.sh OUT
set -u
out=${1:-gpurun_out/kfphase}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/kflag_p1.so indy-plenum_amd/lib/ab/kflag_p3.so indy-plenum_amd/lib/ab/kflag_p6.so; do
  tag=$(basename $lib .so)
  PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/$tag" -o run -- python3 tools/latency.py > "$out/$tag.log" 2>&1 || exit 1
done && \
bash tools/gpu_suite.sh "$out/suite" && \
PV_LAT_CACHED=1 PV_LAT_SIZES=1,16,100,1000,4096 timeout -k 10 200 python3 tools/latency.py > "$out/lat_cached.jsonl" 2>/dev/null && \
PV_LAT_SIZES=1,16,100,1000,4096 timeout -k 10 200 python3 tools/latency.py > "$out/lat_uncached.jsonl" 2>/dev/null && echo done
