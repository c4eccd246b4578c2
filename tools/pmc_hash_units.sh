#!/bin/bash
# PMC passes over k_hash on the C4 shape (1M signatures, 128 B - 4 KB): memory
# pipeline (TA/TD/TCP) busy and stall cycles vs VALU issue, one pass per block
# group (rocprofv3 does not split counters).  bash tools/pmc_hash_units.sh OUTDIR [LIB]
set -u
out=$1; lib=${2:-indy-plenum_amd/lib/libplenum_verify.so}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$tag" -o pmc -- \
    python3 tools/variant_bench.py "$lib" --rounds 1 --n 1000000 --mode 1 --mlen 128 --mlen-max 4096 --cfg 4 \
    --key-mod 1048576 > "$out/$tag.log" 2>&1 || { echo "pass $tag failed"; exit 1; }
  echo "pass $tag ok"
}
run ta TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE GRBM_COUNT
run sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD
run tcp TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES
