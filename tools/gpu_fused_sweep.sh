#!/bin/bash
# Chunking sweep of the fused host-buffer path (C2 end_to_end): chunk count,
# first-chunk size, leading-chunk ramp (PV_HOST_RAMP).
#   bash tools/gpu_fused_sweep.sh OUT
set -u
out=${1:-gpurun_out/fsweep}
mkdir -p "$out"
for k in 1 2 3; do
  for cfg in 8:50:0 8:50:16384 8:50:32768 12:50:16384 6:50:16384 8:50:8192; do
    IFS=: read c p r <<< "$cfg"
    PV_HOST_CHUNKS=$c PV_HOST_FIRST_PCT=$p PV_HOST_RAMP=$r timeout -k 10 300 python bench.py --no-cpu-baseline > "$out/c2_$c.$p.$r.$k.json" 2> "$out/c2_$c.$p.$r.$k.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); e=d['end_to_end']; print(sys.argv[1], d['value'], e['value'], e.get('ms'), e['page_locked_inputs']['value'], e.get('verdict_mismatches'))" "$out/c2_$c.$p.$r.$k.json"
  done
done
