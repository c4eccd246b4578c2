#!/bin/bash
# Interleaved A/B of two builds of libplenum_verify.so on one box (PLENUM_GPU_LIB):
#   bash tools/ab_lib.sh OUT LIB_A LIB_B ROUNDS [bench args...]
# one JSON line per run in OUT/ab.jsonl, tagged with the library.
set -u
out=$1; a=$2; b=$3; rounds=$4; shift 4
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for lib in "$a" "$b"; do
    PLENUM_GPU_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e "$@" > "$out/run.json" 2>> "$out/ab.err" || exit 1
    python - "$lib" "$out/run.json" >> "$out/ab.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'curve_ms': (d.get('kernel_ms') or {}).get('curve'), 'frac': (d.get('roofline') or {}).get('frac')}))
PY
  done
done
cat "$out/ab.jsonl"
