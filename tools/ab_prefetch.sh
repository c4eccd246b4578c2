#!/bin/bash
# A/B of the software-pipelined table reads: default library vs a variant
# built with -D PV_COMB_PREFETCH=0 (keyed comb) -> gpurun_out/ab_pf
set -u
o=gpurun_out/ab_pf; mkdir -p $o
V=${V:-indy-plenum_amd/lib/libpv_nocpf.so}
timeout -k 10 300 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so $V --keyed --rounds 3 --n 4000000 --mode 1 --mlen 128 --mlen-max 4096 --cfg 4 --key-mod 524288 > $o/c4.json 2> $o/c4.err && \
timeout -k 10 300 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so $V --keyed --rounds 5 --n 2500000 --mode 2 --mlen 0 --cfg 3 > $o/c3.json 2> $o/c3.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
echo rc=$?
