#!/bin/bash
# Work-queue chunks sized from the mean message length (PV_HASH_GUIDED=1, the build: ~16 x 64 blocks,
# capped by (indices left) / (2 x waves), 64..1024) against fixed 64-index chunks (lib/ab_chunk64.so) for k_hash
# and k_sha256.  The whole -m gpu suite on the build first, then C3, C4, C2 and
# f3 lines interleaved, two rounds.
#   bash tools/gpu_hash_guided.sh OUT
set -u
out=${1:-gpurun_out/hashguided}
mkdir -p "$out"
echo "[hg] $(date +%T) suite" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || exit 1
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_chunk64.so; do
    tag=$(basename $lib .so)
    echo "[hg] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c3_${tag}_$r.json" 2> "$out/c3_${tag}_$r.err" || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$out/c4_${tag}_$r.json" 2> "$out/c4_${tag}_$r.err" || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-other-configs > "$out/c2_${tag}_$r.json" 2> "$out/c2_${tag}_$r.err" || exit 1
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config f3 --steps 5 --warmup 1 --no-cpu-baseline > "$out/f3_${tag}_$r.json" 2> "$out/f3_${tag}_$r.err" || exit 1
  done
done
echo "[hg] done"
