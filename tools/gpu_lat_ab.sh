#!/bin/bash
# latency check (tools/gpu_lat.sh) + an interleaved C2 curve A/B of library variants
#   bash tools/gpu_lat_ab.sh OUT LIB...
set -u
out=$1; shift
bash tools/gpu_lat.sh "$out" && \
timeout -k 10 400 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so "$@" --rounds 4 > "$out/ab_c2.json" 2> "$out/ab_c2.err"
echo "rc=$?"
