#!/bin/bash
# A/B of the host pipeline's chunking: PV_HOST_CHUNKS x PV_HOST_FIRST_PCT
#   bash tools/gpu_first_chunk.sh OUT
set -u
out=${1:-gpurun_out/first}; mkdir -p "$out"
for c in 8 9 7; do
  for f in 50 100 75; do
    PV_HOST_CHUNKS=$c PV_HOST_FIRST_PCT=$f timeout -k 10 120 python tools/ab_first_chunk.py >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit $?
  done
done
echo rc=0
