#!/bin/bash
# k_hash A/B (hash_ms = k_precheck + k_hash + k_lattice) on C2 and the C4 shape:
#   bash tools/ab_hash2.sh OUTDIR LIB...
set -u
o=$1; shift; mkdir -p $o
timeout -k 10 300 python tools/variant_bench.py "$@" --rounds 4 > $o/c2.json 2> $o/c2.err && \
timeout -k 10 400 python tools/variant_bench.py "$@" --rounds 3 --n 2000000 --mode 1 --mlen 128 --mlen-max 4096 --cfg 4 --key-mod 1048576 > $o/c4.json 2> $o/c4.err && \
timeout -k 10 400 python tools/variant_bench.py "$@" --keyed --rounds 3 --n 2000000 --mode 1 --mlen 128 --mlen-max 4096 --cfg 4 --key-mod 1048576 > $o/c4k.json 2> $o/c4k.err
echo rc=$?
