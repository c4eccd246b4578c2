#!/bin/bash
# First host chunk gathered + DMA'd in 4 pieces (default) vs 1 / 8
# (-D PV_HOST_FIRST_PIECES): host-path tests, then interleaved 1M host-call times.
#   bash tools/gpu_pieces.sh OUT lib_b.so lib_c.so
set -u
out=${1:-gpurun_out/pieces}; shift
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_verify.py -k "host" > "$out/tests.log" 2>&1 && \
PV_HOST_TRACE=1 timeout -k 10 240 python3 tools/e2e_trace.py > "$out/trace.log" 2>&1 && \
bash tools/gpu_e2e_ab.sh "$out" 4 indy-plenum_amd/lib/libplenum_verify.so "$@"
