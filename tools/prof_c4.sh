#!/bin/bash
# rocprofv3 kernel trace of the C4 bench (per-kernel durations incl. k_keys).
set -u
out=${1:-gpurun_out/prof_c4}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --config c4 --steps 2 \
  --warmup 1 --no-cpu-baseline > "$out/prof.log" 2>&1
echo "rc=$?"
