#!/bin/bash
# Upper bound of what key-sorted processing could give C4's keyed curve: the
# same 8M-signature step with the key pool shrunk so every lane's key tables
# stay in L2 (--key-mod 64: lane l of a wave task always uses key l) or in MALL
# (2^13 keys, 76 MB of tables), against the config's 2^20 keys: rocprofv3
# kernel-trace stats of sequential steps, k_curve<true, 0> average.
#   bash tools/gpu_c4_keymod.sh OUT
set -u
out=${1:-gpurun_out/c4km}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for km in 1048576 8192 64; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/km$km" -o run -- python3 bench.py --config c4 --key-mod $km \
      --sequential --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$out/km$km.log" 2>&1 || exit 1
done && echo done
