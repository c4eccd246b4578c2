#!/bin/bash
# Host-buffer pipeline A/B on the GPU box: tools/ab_staging.py per chunk count
# (PV_HOST_CHUNKS is read at pv_init).  bash tools/ab_e2e.sh OUTDIR [chunks...]
set -u
o=$1; shift; mkdir -p $o
for c in "$@"; do PV_HOST_CHUNKS=$c timeout -k 10 200 python tools/ab_staging.py > $o/chunks$c.jsonl 2> $o/chunks$c.err || exit 1; done
echo rc=$?
