#!/bin/bash
# c3bls A/B: the default build against one variant library, interleaved (2 reps),
# then FETCH / WRITE passes of the variant's pair kernel.
#   bash tools/gpu_bls_ab.sh OUT indy-plenum_amd/lib/ab/<variant>.so
set -u
out=${1:-gpurun_out/blsab}; var=$2
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so $var; do
    tag=$(basename $lib .so)
    PLENUM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config c3bls --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls_${tag}_$r.json" 2> "$out/c3bls_${tag}_$r.err" || exit 1
  done
done && \
for c in FETCH_SIZE WRITE_SIZE; do
  PLENUM_GPU_LIB=$var timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$out/pmc/$c" -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --n 500000 --no-cpu-baseline --no-e2e --config c3bls > "$out/pmc_$c.log" 2>&1 || exit 1
done && echo done
