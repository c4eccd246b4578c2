#!/bin/bash
# A/B of k_hash: default library vs $V (C2 and C4 shapes, unkeyed + keyed) -> gpurun_out/ab_hash
set -u
o=gpurun_out/ab_hash; mkdir -p $o
V=${V:-indy-plenum_amd/lib/libpv_oldkeys.so}
timeout -k 10 300 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so $V --rounds 5 > $o/c2.json 2> $o/c2.err && \
timeout -k 10 300 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so $V --keyed --rounds 3 --n 4000000 --mode 1 --mlen 128 --mlen-max 4096 --cfg 4 --key-mod 524288 > $o/c4.json 2> $o/c4.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
echo rc=$?
