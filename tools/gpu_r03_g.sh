#!/bin/bash
# C3 with the enqueue-only tally: tally tests, C3 wide / narrow benches, kernel trace of C3 wide.
set -u
out=${1:-gpurun_out/r03g}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_tally.py tests/test_gpu_device.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > "$out/tests.log" 2>&1 && tail -1 "$out/tests.log" && \
timeout -k 10 240 python bench.py --config c3 --key-format wide > "$out/c3_wide.json" 2> "$out/c3_wide.err" && \
cat "$out/c3_wide.json" && \
timeout -k 10 240 python bench.py --config c3 --key-format narrow > "$out/c3_narrow.json" 2> "$out/c3_narrow.err" && \
cat "$out/c3_narrow.json" && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --config c3 \
    --no-cpu-baseline --no-e2e > "$out/prof.log" 2>&1 && echo done
