#!/bin/bash
# Round-5 roofline evidence for the keyed configs: PMC
# passes (FETCH / WRITE / SQ groups / L2, one group per pass) over the C4 and
# C3 bench lines -- k_keys, k_keys_wide and the keyed curve kernels -- and the
# rocprofv3 kernel-trace stats of the same lines run sequentially.
#   bash tools/gpu_pmc_r05.sh OUT
set -u
out=${1:-gpurun_out/r05pmc}
mkdir -p "$out"
bash tools/pmc_passes.sh "$out/c4" 8000000 --config c4 && \
bash tools/pmc_passes.sh "$out/c3" 2500000 --config c3 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/c4_seq" -o run -- python3 bench.py --config c4 \
    --sequential --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$out/c4_seq.log" 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/c3_seq" -o run -- python3 bench.py --config c3 \
    --sequential --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$out/c3_seq.log" 2>&1 && echo done
