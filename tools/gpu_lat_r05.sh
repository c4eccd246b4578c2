#!/bin/bash
# Round-5 latency evidence: completion-latency microbenchmark (sync / event /
# host poll, default and spin scheduling); kernel durations of the four-side keyed
# kernel with zero-copy and staged inputs; its PV_KEYED_PHASE variants; the -R
# root's split point (PV_ROOT_PRE_SQ = 45 default, 0 / 30 / 60 in lib/ab) as
# kernel durations and interleaved call latencies.
#   bash tools/gpu_lat_r05.sh OUT
set -u
out=${1:-gpurun_out/lat5}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ab=indy-plenum_amd/lib/ab
main=indy-plenum_amd/lib/libplenum_verify.so
timeout -k 10 60 tools/ubench/sync_lat > "$out/sync_default.json" 2>&1 && \
timeout -k 10 60 tools/ubench/sync_lat spin > "$out/sync_spin.json" 2>&1 && \
for zc in default 0; do
  if [ $zc = default ]; then unset PV_SMALL_ZC_MAX; else export PV_SMALL_ZC_MAX=0; fi
  PV_LAT_CACHED=1 PV_LAT_SIZES=1,100 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/zc_$zc" -o run -- python3 tools/latency.py > "$out/zc_$zc.log" 2>&1 || exit 1
done && unset PV_SMALL_ZC_MAX && \
for lib in $ab/keyed_p1.so $ab/keyed_p3.so $ab/keyed_p5.so $ab/keyed_p6.so $ab/root_pre0.so $ab/root_pre30.so $ab/root_pre60.so; do
  tag=$(basename $lib .so)
  PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/$tag" -o run -- python3 tools/latency.py > "$out/$tag.log" 2>&1 || exit 1
done && \
for r in 1 2; do
  for lib in $main $ab/root_pre0.so $ab/root_pre30.so $ab/root_pre60.so; do
    tag=$(basename $lib .so)
    PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1,16,100,1000 timeout -k 10 200 python3 tools/latency.py 2>/dev/null | sed "s/^{/{\"lib\": \"$tag\", \"rep\": $r, /" >> "$out/lat_split.jsonl" || exit 1
  done
done && echo done
