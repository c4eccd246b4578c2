#!/bin/bash
# k_keys with the Montgomery prefix products folded into the stored X and Y
# (lib/ab_keys_xyp.so, -D PV_KEYS_XYP=1: 30 scratch words per entry instead of
# 40, one more multiply per entry) against the build: C4 lines interleaved,
# three rounds, then FETCH_SIZE / WRITE_SIZE passes of a C4 run (2^20 keys) on
# each build.  Also the Merkle GPU tests and f3 lines with the <= 256-node
# one-workgroup tail against per-level launches (lib/ab_no_tail.so).
#   bash tools/gpu_keys_xyp.sh OUT
set -u
out=${1:-gpurun_out/keysxyp}
mkdir -p "$out"
echo "[kx] $(date +%T) merkle tests" && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_merkle.py -m gpu -x -v --timeout 120 --timeout-method thread > "$out/merkle_tests.log" 2>&1 || exit 1
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_keys_xyp.so indy-plenum_amd/lib/ab_no_tail.so; do
    tag=$(basename $lib .so)
    echo "[kx] $(date +%T) $tag $r"
    if [ $tag != ab_no_tail ]; then
      PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$out/c4_${tag}_$r.json" 2> "$out/c4_${tag}_$r.err" || exit 1
    fi
    if [ $tag != ab_keys_xyp ]; then
      PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config f3 --steps 5 --warmup 1 --no-cpu-baseline > "$out/f3_${tag}_$r.json" 2> "$out/f3_${tag}_$r.err" || exit 1
    fi
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_keys_xyp.so; do
  tag=$(basename $lib .so)
  for pass in FETCH_SIZE WRITE_SIZE; do
    echo "[kx] $(date +%T) pmc $tag $pass"
    PLENUM_GPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$out/pmc_$tag/$pass" -o pmc -- \
      python3 bench.py --config c4 --steps 1 --warmup 0 --n 2000000 --no-cpu-baseline --no-e2e > "$out/pmc_${tag}_$pass.log" 2>&1 || exit 1
  done
done
echo "[kx] done"
