#!/bin/bash
# Round-4 roofline evidence on HEAD: PMC passes over the C2 curve kernel
# (FETCH/WRITE in separate passes + SQ groups) and FETCH/WRITE over the C3-BLS
# check kernel, then the rocprofv3 kernel-trace stats of the same bench lines.
#   bash tools/gpu_pmc_r04.sh OUT
set -u
out=${1:-gpurun_out/r04pmc}
mkdir -p "$out"
bash tools/pmc_passes.sh "$out/c2" 1000000 && \
bash tools/pmc_passes.sh "$out/c3bls" 500000 --config c3bls && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_seq" -o run -- python3 bench.py \
    --sequential --no-cpu-baseline --no-e2e > "$out/prof_seq.log" 2>&1 && echo done
