#!/bin/bash
# Lattice stage with carry-chain word arithmetic (device) vs the previous build:
# the -m gpu suite, sequential C2 kernel stats of both, interleaved C2 bench lines
# and 1M host-call times.
#   bash tools/gpu_lattice_ab.sh OUT indy-plenum_amd/lib/ab/head.so
set -u
out=${1:-gpurun_out/latab}; var=$2
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
main=indy-plenum_amd/lib/libplenum_verify.so
bash tools/gpu_suite.sh "$out/suite" && \
for lib in $main $var; do
  tag=$(basename $lib .so)
  PLENUM_GPU_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/seq_$tag" -o run -- python3 bench.py --steps 10 --warmup 3 \
    --sequential --no-cpu-baseline --no-e2e --no-other-configs > "$out/seq_$tag.log" 2>&1 || exit 1
done && \
bash tools/ab_lib.sh "$out/c2" $main $var 3 --no-other-configs && \
bash tools/gpu_e2e_ab.sh "$out/e2e" 3 $main $var
