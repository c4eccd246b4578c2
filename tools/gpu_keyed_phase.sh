#!/bin/bash
# Phase split of k_verify_quad_keyed (cached-key latency kernel): the default
# library against PV_KEYED_PHASE variant builds (1: no -R square root, 2: no
# comb, 3: no hash; wrong verdicts, timing only), host calls of 1 / 100 / 1000
# signatures with every key cached, interleaved:
#   bash tools/gpu_keyed_phase.sh OUT ROUNDS
# (variants built on the CPU first: python indy-plenum_amd/build.py -D PV_KEYED_PHASE=N -o indy-plenum_amd/lib/ab/keyed_pN.so)
set -u
out=$1; rounds=$2
mkdir -p "$out"
libs="indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/keyed_p1.so indy-plenum_amd/lib/ab/keyed_p2.so indy-plenum_amd/lib/ab/keyed_p3.so"
for r in $(seq 1 "$rounds"); do
  for lib in $libs; do
    PLENUM_GPU_LIB=$lib PV_LAT_CACHED=1 PV_LAT_SIZES=1,100,1000 timeout -k 10 200 python tools/latency.py > "$out/lat.tmp" 2>> "$out/lat.err" || exit 1
    python -c "
import json
for l in open('$out/lat.tmp'):
    d = json.loads(l); d['lib'] = '$lib'; print(json.dumps(d))" >> "$out/lat.jsonl" || exit 1
  done
done
cat "$out/lat.jsonl"
