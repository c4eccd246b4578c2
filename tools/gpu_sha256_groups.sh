#!/bin/bash
# k_sha256 with the block window fetched as 4-word groups (<= 5 dwordx4 loads
# per lane and block) and branch-free padding (PV_SHA256_GROUPS=1, the build)
# against 17 guarded dword loads (lib/ab_sha256_words.so, -D PV_SHA256_GROUPS=0):
# the Merkle / SHA-256 GPU tests first, then f3 lines interleaved, three rounds;
# then the C3 / C4 lines of the build (key schedule chosen by the library).
#   bash tools/gpu_sha256_groups.sh OUT
set -u
out=${1:-gpurun_out/sha256groups}
mkdir -p "$out"
echo "[sg] $(date +%T) tests" && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_merkle.py tests/test_gpu_device.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "merkle or sha256 or pipelined" > "$out/tests.log" 2>&1 || exit 1
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_sha256_words.so; do
    tag=$(basename $lib .so)
    echo "[sg] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config f3 --steps 5 --warmup 1 --no-cpu-baseline > "$out/f3_${tag}_$r.json" 2> "$out/f3_${tag}_$r.err" || exit 1
  done
done
echo "[sg] $(date +%T) c3 c4" && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c3.json" 2> "$out/c3.err" && \
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$out/c4.json" 2> "$out/c4.err" && \
echo "[sg] done"
