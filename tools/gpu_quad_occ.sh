#!/bin/bash
# k_verify_quad kernel time vs batch size for LDS-padded variants (blocks per CU capped)
set -u
out=${1:-gpurun_out/occ}; mkdir -p "$out"
L=indy-plenum_amd/lib
for n in 1000 2048 4096 8192 16384 32768; do
  timeout -k 10 120 python tools/variant_bench.py $L/libplenum_verify.so $L/var_pad2.so $L/var_pad1.so --n $n --rounds 8 \
      > "$out/n$n.json" 2> "$out/n$n.err" || exit $?
done
echo rc=0
