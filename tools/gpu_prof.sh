#!/bin/bash
# rocprofv3 kernel stats + PMC passes of the C2 bench only (no e2e calls) -> $1
set -u
out=${1:-gpurun_out/prof}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --no-cpu-baseline --no-e2e \
    > "$out/prof.log" 2>&1 && bash tools/pmc_passes.sh "$out/pmc"
echo rc=$?
