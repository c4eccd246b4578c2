#!/bin/bash
# BLS small-call latency A/B: the BLS GPU tests on the current library, then
# tools/bls_latency.py interleaved over the current and a variant library, and
# one c3bls bench line of each.
#   bash tools/gpu_bls_lat.sh OUT OTHER_LIB
set -u
out=$1; other=$2
cur=indy-plenum_amd/lib/libplenum_verify.so
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_bls_multi.py -x -q --timeout 300 \
    --timeout-method thread > "$out/gpu_tests.log" 2>&1 && tail -1 "$out/gpu_tests.log" && \
for r in 1 2; do
  for lib in $cur $other; do
    PLENUM_GPU_LIB=$lib timeout -k 10 200 python tools/bls_latency.py 1 25 250 2048 8192 > "$out/lat.tmp" 2>> "$out/lat.err" || exit 1
    python -c "
import json, sys
for l in open('$out/lat.tmp'):
    d = json.loads(l); d['lib'] = '$lib'; print(json.dumps(d))" >> "$out/lat.jsonl" || exit 1
  done
done && cat "$out/lat.jsonl" && \
PLENUM_GPU_LIB=$cur timeout -k 10 300 python bench.py --config c3bls --no-cpu-baseline > "$out/c3bls_cur.json" 2> "$out/c3bls.err" && \
PLENUM_GPU_LIB=$other timeout -k 10 300 python bench.py --config c3bls --no-cpu-baseline > "$out/c3bls_other.json" 2>> "$out/c3bls.err" && \
echo done
