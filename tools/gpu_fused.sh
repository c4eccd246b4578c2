#!/bin/bash
# Fused host-buffer chunks (k_chunk_half + k_verify_quad_list) vs the per-chunk
# hash / lattice / curve schedule: GPU tests of the host path, then the C2
# bench line with PV_HOST_FUSED=1 / 0 interleaved (end_to_end is the A/B).
#   bash tools/gpu_fused.sh OUT
set -u
out=${1:-gpurun_out/fused}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py -x -v --timeout 300 --timeout-method thread \
    -k "fused or multi_chunk or page_locked or raw_vectors or adversarial" > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for k in 1 2; do
  for f in 1 0; do
    PV_HOST_FUSED=$f timeout -k 10 300 python bench.py --no-cpu-baseline > "$out/c2_fused$f.$k.json" 2> "$out/c2_fused$f.$k.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); e=d['end_to_end']; print(sys.argv[1], d['value'], e['value'], e.get('ms'), e['page_locked_inputs']['value'], e.get('verdict_mismatches'))" "$out/c2_fused$f.$k.json"
  done
done
