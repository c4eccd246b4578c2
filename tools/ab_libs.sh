#!/bin/bash
# Interleaved A/B/... of several builds of libplenum_verify.so on one box:
#   bash tools/ab_libs.sh OUT ROUNDS "LIB1 LIB2 ..." [bench args...]
# one JSON line per run in OUT/ab.jsonl, tagged with the library.
set -u
out=$1; rounds=$2; libs=$3; shift 3
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for lib in $libs; do
    PLENUM_GPU_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e "$@" > "$out/run.json" 2>> "$out/ab.err" || exit 1
    python - "$lib" "$out/run.json" "$*" >> "$out/ab.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(json.dumps({'lib': sys.argv[1], 'args': sys.argv[3], 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'frac': (d.get('roofline') or {}).get('frac')}))
PY
  done
done
cat "$out/ab.jsonl"
