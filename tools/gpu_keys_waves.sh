#!/bin/bash
# k_keys compiled for 1 / 2 (default) / 3 waves per SIMD: interleaved C4 lines
# (the keyed lines carry roofline.key_prep, k_keys' own HIP-event time).
#   bash tools/gpu_keys_waves.sh OUT lib_a.so lib_b.so ...
set -u
out=$1; shift
mkdir -p "$out"
for r in 1 2; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so "$@"; do
    PLENUM_GPU_LIB=$lib timeout -k 10 400 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
      --no-other-configs > "$out/run.json" 2>> "$out/err.log" || exit 1
    python - "$lib" "$out/run.json" >> "$out/ab.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
kp = d['roofline'].get('key_prep') or {}
print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'keys_ms': kp.get('ms'), 'keys_frac': kp.get('frac'), 'mismatches': d['verdict_mismatches']}))
PY
  done
done
cat "$out/ab.jsonl"
