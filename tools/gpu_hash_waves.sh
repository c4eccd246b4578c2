#!/bin/bash
# k_hash at 4 waves/SIMD (-D PV_HASH_WAVES=4: 128 VGPRs, 76 B of spills) against the
# shipped 3 (148 VGPRs), C4 and C2 lines interleaved, two rounds.
#   bash tools/gpu_hash_waves.sh OUT
set -u
out=${1:-gpurun_out/hashw}
mkdir -p "$out"
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_hash4.so; do
    tag=$(basename $lib .so)
    echo "[hw] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$out/c4_${tag}_$r.json" 2>/dev/null || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-other-configs > "$out/c2_${tag}_$r.json" 2>/dev/null || exit 1
  done
done
echo "[hw] done"
