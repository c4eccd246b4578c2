#!/bin/bash
# BLS small-call latency of several library builds, interleaved:
#   bash tools/gpu_lat_libs.sh OUT ROUNDS "LIB1 LIB2 ..." [sizes...]
set -u
out=$1; rounds=$2; libs=$3; shift 3
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for lib in $libs; do
    PLENUM_GPU_LIB=$lib timeout -k 10 200 python tools/bls_latency.py "$@" > "$out/lat.tmp" 2>> "$out/lat.err" || exit 1
    python -c "
import json
for l in open('$out/lat.tmp'):
    d = json.loads(l); d['lib'] = '$lib'; print(json.dumps(d))" >> "$out/lat.jsonl" || exit 1
  done
done
cat "$out/lat.jsonl"
