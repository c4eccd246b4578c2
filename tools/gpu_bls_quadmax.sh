#!/bin/bash
# Lane-quad vs lane-pair BLS kernel by call size after the quad final
# exponentiation: bls_latency.py over a pair-only (-D PV_BLS_QUAD_MAX=0) and a
# quad-always build, then the c3bls bench line of the quad-always build.
#   bash tools/gpu_bls_quadmax.sh OUT PAIR_LIB QUAD_LIB
set -u
out=$1; pair=$2; quad=$3
mkdir -p "$out"
for lib in $pair $quad; do
  PLENUM_GPU_LIB=$lib timeout -k 10 300 python tools/bls_latency.py 2048 8192 16384 32768 65536 > "$out/lat.tmp" 2>> "$out/lat.err" || exit 1
  python -c "
import json
for l in open('$out/lat.tmp'):
    d = json.loads(l); d['lib'] = '$lib'; print(json.dumps(d))" >> "$out/lat.jsonl" || exit 1
done
cat "$out/lat.jsonl"
PLENUM_GPU_LIB=$quad timeout -k 10 300 python bench.py --config c3bls --no-cpu-baseline > "$out/c3bls_quad.json" 2> "$out/c3bls.err" && \
PLENUM_GPU_LIB=$pair timeout -k 10 300 python bench.py --config c3bls --no-cpu-baseline > "$out/c3bls_pair.json" 2>> "$out/c3bls.err" && \
tail -c 300 "$out/c3bls_quad.json" && echo && tail -c 300 "$out/c3bls_pair.json" && echo done
