#!/bin/bash
# One rocprofv3 PMC pass (SQ counters) over the C4 bench: instruction mix and
# stall composition of k_hash / keyed k_curve.  Run on the GPU box.
set -u
out=${1:-gpurun_out/pmc_c4}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d "$out/sq" -o pmc -- \
  python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > "$out/sq.log" 2>&1
echo "pass sq rc=$?"
