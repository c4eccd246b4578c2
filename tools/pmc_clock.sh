#!/bin/bash
# GPU clock during the C2 curve kernel: GRBM_GUI_ACTIVE (GPU cycles, summed over
# XCDs) against the dispatch's own start/end timestamps in the same CSV.
#   bash tools/pmc_clock.sh OUTDIR LIB...      (on the GPU box)
set -u
out=$1; shift; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  PLENUM_GPU_LIB=$(realpath "$lib") timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES \
      --output-format csv -d "$out/$tag" -o pmc -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$out/$tag.log" 2>&1 || exit 1
  echo "pass $tag ok"
done
