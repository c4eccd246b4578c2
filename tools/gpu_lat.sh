#!/bin/bash
# Latency-kernel check on the GPU box: the curve-mode / small-batch parity
# tests, the host-buffer latency sweep with the lane-quad kernel (default) and
# the lane-pair kernel (A/B), and a rocprofv3 kernel trace of the quad sweep.
#   bash tools/gpu_lat.sh gpurun_out/lat
set -u
out=${1:-gpurun_out/lat}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_device.py -x -v --timeout 300 --timeout-method thread \
    -k "curve_modes or latency_kernel" > "$out/tests.log" 2>&1 && tail -2 "$out/tests.log" && \
timeout -k 10 200 python tools/latency.py > "$out/latency_quad.jsonl" 2> "$out/latency_quad.err" && \
PV_LAT_KERNEL=pair timeout -k 10 200 python tools/latency.py > "$out/latency_pair.jsonl" 2> "$out/latency_pair.err" && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 tools/latency.py \
    > "$out/prof.log" 2>&1
echo "rc=$?"
