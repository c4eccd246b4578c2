#!/bin/bash
# SQ instruction counters of the C2 curve kernel for library variants, one
# rocprofv3 --pmc pass per variant (MI355X_MICROARCH.md rocprofv3 section).
#   bash tools/pmc_ab.sh OUTDIR LIB...      (on the GPU box)
set -u
out=$1; shift; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  PLENUM_GPU_LIB=$(realpath "$lib") timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU \
      SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
      --output-format csv -d "$out/$tag" -o pmc -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > "$out/$tag.log" 2>&1 || exit 1
  echo "pass $tag ok"
done
