#!/bin/bash
# Key preparation beside the hash stage (pv_verify_keys_device_async: k_keys /
# k_keys_wide on the slot's side stream while k_hash runs) against the serial
# schedule (--keys-serial: keys, then hash, on the step's stream).  First the
# pipelined-slot GPU tests, then C4 and C3 lines interleaved, three rounds.
#   bash tools/gpu_keys_beside.sh OUT
set -u
out=${1:-gpurun_out/keysbeside}
mkdir -p "$out"
echo "[kb] $(date +%T) tests" && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_device.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "pipelined" > "$out/tests.log" 2>&1 || exit 1
for r in 1 2 3; do
  for mode in beside serial; do
    flag=""
    [ $mode = serial ] && flag="--keys-serial"
    echo "[kb] $(date +%T) $mode $r"
    timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline $flag > "$out/c4_${mode}_$r.json" 2> "$out/c4_${mode}_$r.err" || exit 1
    timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $flag > "$out/c3_${mode}_$r.json" 2> "$out/c3_${mode}_$r.err" || exit 1
  done
done
echo "[kb] done"
