#!/bin/bash
# Full -m gpu suite, the latency sweep, a phase split of the one-launch latency
# kernel (variant libs with PV_QUAD_PHASE=1/2/3, n = 1000 device-resident) and
# the host-buffer staging sweep (chunks x gather threads).
#   bash tools/gpu_suite_e2e.sh OUT
set -u
out=${1:-gpurun_out/suite}
mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 200 python tools/latency.py > "$out/latency.jsonl" 2> "$out/latency.err" || exit $?
L=indy-plenum_amd/lib
timeout -k 10 300 python tools/variant_bench.py $L/libplenum_verify.so $L/var_phase1.so $L/var_phase2.so $L/var_phase3.so \
    --n 1000 --rounds 20 --no-check > "$out/quad_phases.json" 2> "$out/quad_phases.err" || exit $?
for c in 6 8 10; do
  PV_HOST_CHUNKS=$c timeout -k 10 200 python tools/ab_staging.py > "$out/staging_c$c.jsonl" 2> "$out/staging_c$c.err" || exit $?
done
echo "rc=0"
