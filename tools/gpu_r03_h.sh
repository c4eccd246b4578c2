#!/bin/bash
# sliced wide key preparation: key-cache / device tests, C3 wide bench, kernel trace
set -u
out=${1:-gpurun_out/r03h}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_device.py tests/test_gpu_c1.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 && tail -1 "$out/tests.log" && \
timeout -k 10 240 python bench.py --config c3 > "$out/c3_wide.json" 2> "$out/c3_wide.err" && cat "$out/c3_wide.json" && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --config c3 \
    --no-cpu-baseline --no-e2e > "$out/prof.log" 2>&1 && echo done
