#!/bin/bash
# Deferred-record pass overlapping the last chunk (k_verify_quad_stream) vs one
# pass after it (-D PV_DEFER_STREAM=0): host-path tests, kernel timeline of the
# new build, interleaved 1M host-call times.
#   bash tools/gpu_defer_stream.sh OUT indy-plenum_amd/lib/ab/defer_after.so
set -u
out=${1:-gpurun_out/dstream}; var=$2
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
main=indy-plenum_amd/lib/libplenum_verify.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_verify.py -k "host_fused or defer_stream" > "$out/tests.log" 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 tools/e2e_trace.py > "$out/prof.log" 2>&1 && \
for r in 1 2 3; do
  for lib in $main $var; do
    PLENUM_GPU_LIB=$lib timeout -k 10 240 python3 tools/e2e_calls.py 8 >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit 1
  done
done && echo done
