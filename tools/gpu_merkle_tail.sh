#!/bin/bash
# The -m gpu suite on the build, then f3 lines with the one-workgroup Merkle
# tail (k_merkle_tail for the last <= 2048 nodes, the build) against one
# k_merkle_level launch per level (lib/ab_no_tail.so), three rounds
# interleaved; then the C3 / C4 / C2 lines of the build.
#   bash tools/gpu_merkle_tail.sh OUT
set -u
out=${1:-gpurun_out/merkletail}
mkdir -p "$out"
echo "[mt] $(date +%T) suite" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || exit 1
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_no_tail.so; do
    tag=$(basename $lib .so)
    echo "[mt] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config f3 --steps 5 --warmup 1 --no-cpu-baseline > "$out/f3_${tag}_$r.json" 2> "$out/f3_${tag}_$r.err" || exit 1
  done
done
echo "[mt] $(date +%T) lines" && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c3.json" 2> "$out/c3.err" && \
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$out/c4.json" 2> "$out/c4.err" && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-other-configs > "$out/c2.json" 2> "$out/c2.err" && \
echo "[mt] done"
