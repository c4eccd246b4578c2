#!/bin/bash
# page-locked inputs: round-sized chunks (default) vs gather-sized chunks (PV_HOST_ROUNDS=0)
set -u
out=${1:-gpurun_out/locked}; mkdir -p "$out"
for r in 1 2; do
  for hr in 1 0; do
    PV_HOST_ROUNDS=$hr timeout -k 10 120 python tools/ab_locked.py >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit $?
  done
done
echo rc=0
