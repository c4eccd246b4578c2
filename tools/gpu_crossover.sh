#!/bin/bash
# Latency-kernel / fused-chunk crossover of pv_verify_batch (host buffers):
# k_verify_quad (PV_LAT_MAX large) vs the chunk path (PV_LAT_MAX=0, fused
# chunks) at sizes around the default PV_LAT_MAX.   bash tools/gpu_crossover.sh OUT
set -u
out=${1:-gpurun_out/xover}
mkdir -p "$out"
S=4096,8192,16384,24576,32768,49152,65536,131072
PV_LAT_SIZES=$S PV_LAT_MAX=1048576 timeout -k 10 200 python tools/latency.py > "$out/quad.jsonl" 2> "$out/quad.err" || exit 1
PV_LAT_SIZES=$S PV_LAT_MAX=0 timeout -k 10 200 python tools/latency.py > "$out/fused.jsonl" 2> "$out/fused.err" || exit 1
PV_LAT_SIZES=$S PV_LAT_MAX=0 PV_HOST_FUSED=0 timeout -k 10 200 python tools/latency.py > "$out/unfused.jsonl" 2> "$out/unfused.err" || exit 1
paste <(python -c "import json;[print(json.loads(l)['n'], json.loads(l)['ms_median']) for l in open('$out/quad.jsonl')]") \
      <(python -c "import json;[print(json.loads(l)['ms_median']) for l in open('$out/fused.jsonl')]") \
      <(python -c "import json;[print(json.loads(l)['ms_median']) for l in open('$out/unfused.jsonl')]")
