#!/bin/bash
# Interleaved A/B of library variants (tools/variant_bench.py) on C2 and the
# keyed C3 path.  Usage on the GPU box: bash tools/ab_variants.sh OUTDIR LIB...
set -u
o=$1; shift; mkdir -p $o
timeout -k 10 400 python tools/variant_bench.py "$@" --rounds 4 > $o/c2.json 2> $o/c2.err && \
timeout -k 10 300 python tools/variant_bench.py "$@" --keyed --rounds 3 --n 2500000 --mode 2 --mlen 0 --cfg 3 > $o/c3.json 2> $o/c3.err
echo rc=$?
