#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C2 bench for library variants:
#   bash tools/stats_ab.sh OUTDIR LIB...
set -u
out=$1; shift; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  PLENUM_GPU_LIB=$(realpath "$lib") timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/$tag" -o run -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$out/$tag.log" 2>&1 || exit 1
  echo "pass $tag ok"
done
