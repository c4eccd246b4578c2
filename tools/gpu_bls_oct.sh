#!/bin/bash
# Lane-octet BLS kernel: the BLS GPU tests, then tools/bls_latency.py interleaved
# with the octet forced (PV_BLS_OCT_MAX=1048576), the quad (PV_BLS_OCT_MAX=0) and
# the pair (both 0) kernels, and the c3bls bench line.
#   bash tools/gpu_bls_oct.sh OUT
set -u
out=$1
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_bls_multi.py -x -q --timeout 300 \
    --timeout-method thread > "$out/gpu_tests.log" 2>&1 && tail -1 "$out/gpu_tests.log" || exit 1
for r in 1 2; do
  for cfg in "1048576 32768 oct" "0 32768 quad" "0 0 pair"; do
    set -- $cfg
    PV_BLS_OCT_MAX=$1 PV_BLS_QUAD_MAX=$2 timeout -k 10 200 python tools/bls_latency.py 1 25 250 2048 8192 16384 \
        > "$out/lat.tmp" 2>> "$out/lat.err" || exit 1
    python -c "
import json
for l in open('$out/lat.tmp'):
    d = json.loads(l); d['kernel'] = '$3'; print(json.dumps(d))" >> "$out/lat.jsonl" || exit 1
  done
done
cat "$out/lat.jsonl"
timeout -k 10 300 python bench.py --config c3bls --no-cpu-baseline > "$out/c3bls.json" 2> "$out/c3bls.err" && \
tail -c 250 "$out/c3bls.json" && echo && echo done
