#!/bin/bash
# PMC passes over the c3bls check kernel for two library builds (the shipped
# lane-pair kernel and the one-lane variant lib/ab/one_lane.so): issue, wait,
# instruction-cache and LDS counters, one counter group per rocprofv3 pass.
#   bash tools/gpu_bls_pmc_ab.sh OUT
set -u
out=${1:-gpurun_out/bls_pmc_ab}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  lib=$1; tag=$2; shift 2
  PLENUM_GPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$tag" -o pmc -- \
    python3 bench.py --config c3bls --steps 1 --warmup 0 --n 500000 --no-cpu-baseline > "$out/$tag.log" 2>&1
  rc=$?
  echo "[pmc] $(date +%T) $tag rc=$rc"
  return $rc
}
for v in pair:indy-plenum_amd/lib/libplenum_verify.so one:indy-plenum_amd/lib/ab/one_lane.so; do
  t=${v%%:*}; lib=${v#*:}
  run "$lib" "${t}_sq1" SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS || exit 1
  run "$lib" "${t}_sq2" SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS SQ_IFETCH GRBM_GUI_ACTIVE || exit 1
  run "$lib" "${t}_ic" SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit 1
  run "$lib" "${t}_fetch" FETCH_SIZE || exit 1
  run "$lib" "${t}_write" WRITE_SIZE || exit 1
done
echo "[pmc] done"
