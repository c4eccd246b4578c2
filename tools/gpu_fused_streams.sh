#!/bin/bash
# Fused host chunks over 2 vs 3 compute streams, with ramps starting at 8k /
# 16k / 32k signatures (C2 end_to_end, interleaved).  bash tools/gpu_fused_streams.sh OUT
# (PV_HOST_STREAMS was removed after this A/B: profiles/r02_ab_fused_streams_notadopted.jsonl)
set -u
out=${1:-gpurun_out/fstreams}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -q --timeout 200 --timeout-method thread \
    -k "fused or multi_chunk" > "$out/tests.log" 2>&1 || { tail -20 "$out/tests.log"; exit 1; }
PV_HOST_STREAMS=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -q --timeout 200 --timeout-method thread \
    -k "fused or multi_chunk" >> "$out/tests.log" 2>&1 || { tail -20 "$out/tests.log"; exit 1; }
grep passed "$out/tests.log"
for k in 1 2 3; do
  for cfg in 2:32768 3:32768 3:16384 3:8192 2:16384; do
    IFS=: read st r <<< "$cfg"
    PV_HOST_STREAMS=$st PV_HOST_RAMP=$r timeout -k 10 300 python bench.py --no-cpu-baseline > "$out/c2_$st.$r.$k.json" 2> "$out/c2_$st.$r.$k.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); e=d['end_to_end']; print(sys.argv[1], d['value'], e['value'], e.get('ms'), e['page_locked_inputs']['value'], e.get('verdict_mismatches'))" "$out/c2_$st.$r.$k.json"
  done
done
