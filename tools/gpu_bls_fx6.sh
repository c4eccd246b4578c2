#!/bin/bash
# Round 6: the pair kernel's final exponentiation as a step
# program whose product streams its first operand from the LDS slot.  GPU ==
# oracle BLS tests, the c3bls line interleaved against the chain-of-calls build
# (indy-plenum_amd/lib/ab_fe_chain.so: -D PV_FE_PROG=0), FETCH / WRITE passes.
#   bash tools/gpu_bls_fx6.sh OUT
set -u
out=${1:-gpurun_out/blsfx6}
mkdir -p "$out"
echo "[fx6] $(date +%T) tests" && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bls.py tests/test_gpu_bls_multi.py > "$out/tests.log" 2>&1 && \
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_fe_chain.so; do
    tag=$(basename $lib .so)
    echo "[fx6] $(date +%T) bench $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls_${tag}_$r.json" 2> "$out/c3bls_${tag}_$r.err" || exit 1
  done
done && \
echo "[fx6] $(date +%T) pmc" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$out/pmc/$c" -o pmc -- \
    python3 bench.py --config c3bls --steps 1 --warmup 0 --n 500000 --no-cpu-baseline > "$out/pmc_$c.log" 2>&1 || exit 1
  echo "[fx6] pass $c ok"
done && echo "[fx6] done"
