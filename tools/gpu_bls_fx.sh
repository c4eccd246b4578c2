#!/bin/bash
# BLS final exponentiation as a step program (round 5): GPU == oracle tests, the
# c3bls line interleaved against the out-of-line build (lib/ab/fe_calls.so), lone-
# check latency, PMC passes and kernel stats of the new build.
#   bash tools/gpu_bls_fx.sh OUT
set -u
out=${1:-gpurun_out/blsfx}
mkdir -p "$out"
echo "[fx] $(date +%T) tests" && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bls.py tests/test_gpu_bls_multi.py > "$out/tests.log" 2>&1 && \
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/fe_calls.so; do
    tag=$(basename $lib .so)
    echo "[fx] $(date +%T) bench $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls_${tag}_$r.json" 2> "$out/c3bls_${tag}_$r.err" || exit 1
  done
done && \
echo "[fx] $(date +%T) pmc" && \
bash tools/pmc_passes.sh "$out/pmc" 500000 --config c3bls && \
echo "[fx] $(date +%T) stats" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --config c3bls \
    --steps 3 --warmup 1 --no-cpu-baseline > "$out/prof.log" 2>&1 && echo "[fx] done"
