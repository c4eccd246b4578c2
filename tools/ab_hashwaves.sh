#!/bin/bash
# k_hash occupancy A/B: 4 waves/SIMD (default, 116 VGPRs) vs forced 5 and 6 -> gpurun_out/ab_hw
set -u
o=gpurun_out/ab_hw; mkdir -p $o
L=indy-plenum_amd/lib
timeout -k 10 300 python tools/variant_bench.py $L/libplenum_verify.so $L/libpv_hw5.so $L/libpv_hw6.so --keyed --rounds 3 --n 4000000 --mode 1 --mlen 128 --mlen-max 4096 --cfg 4 --key-mod 524288 > $o/c4.json 2> $o/c4.err
echo rc=$?
