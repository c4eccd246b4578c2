#!/bin/bash
# rocprofv3 PMC passes over the C2 bench (one counter group per pass, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes).  Run on the GPU box:
#   bash tools/pmc_passes.sh <outdir> [n] [extra bench.py args, e.g. --config c3bls]
set -u
out=${1:-gpurun_out/pmc}; n=${2:-1000000}; shift 2 2>/dev/null; extra=("$@")
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$tag" -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --n "$n" --no-cpu-baseline --no-e2e "${extra[@]}" > "$out/$tag.log" 2>&1
  rc=$?
  echo "pass $tag rc=$rc"
  return $rc
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS && \
run sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT && \
run l2 TCC_HIT_sum TCC_MISS_sum
