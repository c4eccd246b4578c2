#!/bin/bash
# The -m gpu suite and smoke() on the current build (log per step under OUT).
#   bash tools/gpu_suite.sh OUT
set -u
out=${1:-gpurun_out/suite}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 && echo suite-ok
