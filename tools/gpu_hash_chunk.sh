#!/bin/bash
# Work-queue chunk size of k_hash / k_sha256 (indices per wave atomic on the one
# global counter): 64 (the build) against 256 and 1024 (-D PV_HASH_CHUNK=...),
# C3 (one-block messages: one atomic per wave per trip at 64), C4, C2 and f3
# lines interleaved, two rounds.
#   bash tools/gpu_hash_chunk.sh OUT
set -u
out=${1:-gpurun_out/hashchunk}
mkdir -p "$out"
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_chunk256.so indy-plenum_amd/lib/ab_chunk1024.so; do
    tag=$(basename $lib .so)
    echo "[hc] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c3_${tag}_$r.json" 2> "$out/c3_${tag}_$r.err" || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$out/c4_${tag}_$r.json" 2> "$out/c4_${tag}_$r.err" || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-other-configs > "$out/c2_${tag}_$r.json" 2> "$out/c2_${tag}_$r.err" || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config f3 --steps 5 --warmup 1 --no-cpu-baseline > "$out/f3_${tag}_$r.json" 2> "$out/f3_${tag}_$r.err" || exit 1
  done
done
echo "[hc] done"
