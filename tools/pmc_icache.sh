#!/bin/bash
# Instruction-cache PMC of the curve kernels: C2 bench (k_curve_half) and the
# latency sweep at n = 1000 / 2048 (k_verify_quad).  bash tools/pmc_icache.sh OUT
set -u
out=${1:-gpurun_out/icache}; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_TC_INST_REQ"
timeout -s KILL 90 rocprofv3 --pmc $C SQ_IFETCH SQ_WAVES --output-format csv -d "$out/c2" -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > "$out/c2.log" 2>&1 && echo c2 ok && \
PV_LAT_SIZES=1000,2048 timeout -s KILL 90 rocprofv3 --pmc $C SQ_IFETCH SQ_WAVES --output-format csv -d "$out/lat" -o pmc -- \
    python3 tools/latency.py > "$out/lat.log" 2>&1 && echo lat ok
