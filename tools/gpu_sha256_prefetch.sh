#!/bin/bash
# k_sha256 with each lane's next block window loaded one trip ahead (default)
# against loading it right before the compression (-D PV_SHA256_PREFETCH=0):
# the Merkle GPU tests, then the f3 line interleaved, three rounds.
#   bash tools/gpu_sha256_prefetch.sh OUT
set -u
out=${1:-gpurun_out/shapf}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_merkle.py > "$out/tests.log" 2>&1 || exit 1
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_sha_noprefetch.so; do
    tag=$(basename $lib .so)
    PLENUM_GPU_LIB=$lib timeout -k 10 200 python bench.py --config f3 --steps 5 --warmup 1 > "$out/f3_${tag}_$r.json" 2>/dev/null || exit 1
  done
done
echo done
