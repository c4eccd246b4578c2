#!/bin/bash
# Full -m gpu suite, then the host-buffer staging sweep (chunks x gather threads).
#   bash tools/gpu_suite_e2e.sh OUT
set -u
out=${1:-gpurun_out/suite}
mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
for c in 6 8 10; do
  PV_HOST_CHUNKS=$c timeout -k 10 200 python tools/ab_staging.py > "$out/staging_c$c.jsonl" 2> "$out/staging_c$c.err" || exit $?
done
echo "rc=0"
