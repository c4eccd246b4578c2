#!/bin/bash
# Generic latency A/B: the default build against one variant library: the -m gpu
# suite (default build), kernel-trace stats of a lone cached call for both, and
# interleaved host-call latencies (cached keys; uncached too with UNCACHED=1).
#   bash tools/gpu_lat_ab.sh OUT indy-plenum_amd/lib/ab/<variant>.so
set -u
out=${1:-gpurun_out/latab}; var=$2
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
main=indy-plenum_amd/lib/libplenum_verify.so
bash tools/gpu_suite.sh "$out/suite" && \
for lib in $main $var; do
  tag=$(basename $lib .so)
  PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1,100 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof_$tag" -o run -- python3 tools/latency.py > "$out/prof_$tag.log" 2>&1 || exit 1
done && \
for r in 1 2 3; do
  for lib in $main $var; do
    tag=$(basename $lib .so)
    for c in 1 ${UNCACHED:+0}; do
      PLENUM_GPU_LIB=$lib PV_LAT_CACHED=$c PV_LAT_SIZES=1,16,100,1000,4096 timeout -k 10 200 python3 tools/latency.py 2>/dev/null | sed "s/^{/{\"lib\": \"$tag\", \"rep\": $r, /" >> "$out/lat_ab.jsonl" || exit 1
    done
  done
done && echo done
