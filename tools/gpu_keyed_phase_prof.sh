#!/bin/bash
# Kernel durations (rocprofv3 --kernel-trace --stats) of the cached-key latency
# kernel at 1 and 1000 signatures per call, default build and PV_KEYED_PHASE
# variants (PV_KEYED_PHASE bit mask: 1 no -R root, 2 no comb, 4 no hash):
#   bash tools/gpu_keyed_phase_prof.sh OUT
set -u
out=$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/keyed_p1.so indy-plenum_amd/lib/ab/keyed_p2.so indy-plenum_amd/lib/ab/keyed_p4.so indy-plenum_amd/lib/ab/keyed_p3.so indy-plenum_amd/lib/ab/keyed_p5.so indy-plenum_amd/lib/ab/keyed_p6.so indy-plenum_amd/lib/ab/keyed_p7.so; do
  tag=$(basename $lib .so)
  for n in 1 1000; do
    PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=$n timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/${tag}_$n" -o run -- python3 tools/latency.py > "$out/${tag}_$n.log" 2>&1 || exit 1
  done
done
echo done
