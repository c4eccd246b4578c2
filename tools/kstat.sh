#!/bin/bash
# Register / scratch / occupancy of every kernel in pv_kernels.hip (gfx950),
# from a device-only -S compile.  Usage: tools/kstat.sh [-DFOO ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
out=${KSTAT_OUT:-/tmp/pv_kernels.s}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I$R/include "$@" -x hip --cuda-device-only -S \
  $R/indy-plenum_amd/csrc/pv_kernels.hip -o $out 2>/dev/null
awk '/\.amdhsa_kernel /{k=$2} /; NumVgprs:/{v=$3} /; ScratchSize:/{s=$3} /; Occupancy:/{printf "%-60s vgpr %4s scratch %4s occ %s\n", k, v, s, $3}' $out
