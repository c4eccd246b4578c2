#!/bin/bash
# k_hash with the first 2 or 4 16-byte groups of the next block's message window
# loaded one compression ahead (-D PV_HASH_PF=2 / 4, still 3 waves/SIMD) against
# none (the shipped build at the time), C4 and C2 lines interleaved, two rounds.
#   bash tools/gpu_hash_pf.sh OUT
set -u
out=${1:-gpurun_out/hashpf}
mkdir -p "$out"
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_hashpf2.so indy-plenum_amd/lib/ab_hashpf4.so; do
    tag=$(basename $lib .so)
    echo "[pf] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$out/c4_${tag}_$r.json" 2>/dev/null || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-other-configs > "$out/c2_${tag}_$r.json" 2>/dev/null || exit 1
  done
done
echo "[pf] done"
