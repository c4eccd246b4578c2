#!/bin/bash
# Instruction-cache PMC of the cached-key latency kernel (k_verify_quad_keyed:
# three waves running three different code paths -- hash, comb, square root)
# and the uncached one (k_verify_quad), host calls of 1 and 1000 signatures.
#   bash tools/pmc_icache_keyed.sh OUT
set -u
out=${1:-gpurun_out/icache_keyed}; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_TC_INST_REQ"
PV_LAT_CACHED=1 PV_LAT_SIZES=1,1000 timeout -s KILL 90 rocprofv3 --pmc $C SQ_IFETCH SQ_WAVES --output-format csv \
    -d "$out/keyed" -o pmc -- python3 tools/latency.py > "$out/keyed.log" 2>&1 && echo keyed ok && \
PV_LAT_SIZES=1,1000 timeout -s KILL 90 rocprofv3 --pmc $C SQ_IFETCH SQ_WAVES --output-format csv \
    -d "$out/quad" -o pmc -- python3 tools/latency.py > "$out/quad.log" 2>&1 && echo quad ok
