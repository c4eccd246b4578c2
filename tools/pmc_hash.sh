#!/bin/bash
# SQ counters of k_hash on the C4 shape (ragged 128 B - 4 KB, key pool): one
# rocprofv3 --pmc pass per counter group.  bash tools/pmc_hash.sh OUTDIR [n]
set -u
out=$1; n=${2:-2000000}; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$tag" -o pmc -- \
    python3 bench.py --config c4 --steps 1 --warmup 0 --n "$n" --no-cpu-baseline --no-e2e > "$out/$tag.log" 2>&1
  rc=$?; echo "pass $tag rc=$rc"; return $rc
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD && \
run mem FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum && \
run clk GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
