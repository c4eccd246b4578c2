#!/bin/bash
# HBM traffic of the C2 curve kernel per library variant (FETCH_SIZE and
# WRITE_SIZE passes over tools/variant_bench.py, one library per process):
#   bash tools/pmc_traffic_ab.sh OUTDIR LIB...
set -u
o=$1; shift; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  tag=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE TCC_HIT_sum; do
    extra=""; [ $c = TCC_HIT_sum ] && extra="TCC_MISS_sum"
    timeout -s KILL 120 rocprofv3 --pmc $c $extra --output-format csv -d $o/$tag/$c -o pmc -- \
      python3 tools/variant_bench.py $lib --rounds 1 > $o/$tag.$c.log 2>&1 || { echo "pass $tag $c failed"; exit 1; }
  done
  echo "pass $tag ok"
done
