#!/bin/bash
# GPU parity round: smoke(), then the given test files (default: the whole -m gpu suite).
#   bash tools/gpu_tests.sh OUT [pytest args...]
set -u
out=${1:-gpurun_out/tests}
shift || true
mkdir -p "$out"
args=${*:-tests}
echo "[gpu_tests] $(date +%T) smoke" && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 && \
tail -1 "$out/smoke.log" && echo "[gpu_tests] $(date +%T) pytest $args" && \
timeout -k 10 900 python -u -m pytest $args -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
exit $rc
