#!/bin/bash
# Narrow prepared-key format A/B: the -m gpu suite on the current library, then
# interleaved C4 / C1 bench runs and the cached-key latency sweep against a
# variant library (e.g. one built from the previous commit's sources).
#   bash tools/gpu_kfmt_ab.sh OUT OTHER_LIB
set -u
out=$1; other=$2
cur=indy-plenum_amd/lib/libplenum_verify.so
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 && tail -1 "$out/gpu_tests.log" && \
bash tools/ab_libs.sh "$out/c4" 3 "$cur $other" --config c4 --steps 5 --warmup 2 && \
bash tools/ab_libs.sh "$out/c1" 2 "$cur $other" --config c1 && \
PV_LAT_CACHED=1 timeout -k 10 240 python tools/latency.py > "$out/lat_cached_cur.jsonl" 2> "$out/lat.err" && \
PLENUM_GPU_LIB="$other" PV_LAT_CACHED=1 timeout -k 10 240 python tools/latency.py > "$out/lat_cached_other.jsonl" 2>> "$out/lat.err" && \
echo done
