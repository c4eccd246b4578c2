#!/bin/bash
# Interleaved 1M host-call times (tools/e2e_calls.py) of several library builds:
#   bash tools/gpu_e2e_ab.sh OUT ROUNDS lib1.so lib2.so ...
set -u
out=$1; rounds=$2; shift 2
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    PLENUM_GPU_LIB=$lib timeout -k 10 240 python3 tools/e2e_calls.py 10 >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit 1
  done
done && echo done
