#!/bin/bash
# First host chunk read in place (mapped page-locked memory) vs after its DMA
# (-D PV_HOST_ZC_FIRST=0): host-path tests, then interleaved 1M host-call times.
#   bash tools/gpu_zc_first.sh OUT indy-plenum_amd/lib/ab/zcfirst_off.so
set -u
out=${1:-gpurun_out/zcfirst}; var=$2
mkdir -p "$out"
main=indy-plenum_amd/lib/libplenum_verify.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_verify.py -k "host_fused or first_chunk" > "$out/tests.log" 2>&1 && \
PV_HOST_TRACE=1 timeout -k 10 240 python3 tools/e2e_trace.py > "$out/trace.log" 2>&1 && \
bash tools/gpu_e2e_ab.sh "$out" 4 $main $var
