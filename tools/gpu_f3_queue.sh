#!/bin/bash
# f3 lines (k_sha256 leaf kernel) of three work-queue builds interleaved, three
# rounds: the build (chunks from the mean message length), chunks capped only by
# what is left (lib/ab_sha_fit1024.so) and fixed 64 (lib/ab_chunk64.so); then
# C3 / C2 lines of the build.
#   bash tools/gpu_f3_queue.sh OUT
set -u
out=${1:-gpurun_out/f3queue}
mkdir -p "$out"
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_sha_fit1024.so indy-plenum_amd/lib/ab_chunk64.so; do
    tag=$(basename $lib .so)
    echo "[fq] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config f3 --steps 5 --warmup 1 --no-cpu-baseline > "$out/f3_${tag}_$r.json" 2> "$out/f3_${tag}_$r.err" || exit 1
  done
done
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c3.json" 2> "$out/c3.err" && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-other-configs > "$out/c2.json" 2> "$out/c2.err" && \
echo "[fq] done"
