#!/bin/bash
# Leading-chunk ramp x chunk count of the fused host-buffer path on the round-5
# build (C2 end_to_end of bench.py, other configs off), two interleaved reps.
#   bash tools/gpu_ramp_sweep.sh OUT
set -u
out=${1:-gpurun_out/ramp}
mkdir -p "$out"
for k in 1 2; do
  for cfg in 8:32768 8:16384 8:8192 12:16384 12:32768 6:32768; do
    IFS=: read c r <<< "$cfg"
    PV_HOST_CHUNKS=$c PV_HOST_RAMP=$r timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-configs --steps 5 --warmup 2 > "$out/c2_$c.$r.$k.json" 2> "$out/c2_$c.$r.$k.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); e=d['end_to_end']; print(sys.argv[1], d['value'], e['value'], e.get('ms'), e['page_locked_inputs']['value'])" "$out/c2_$c.$r.$k.json" >> "$out/summary.txt"
  done
done && echo done
