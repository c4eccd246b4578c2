#!/bin/bash
# GPU check after a kernel change: -m gpu suite, then the c2 / c4 / f3 bench lines.
#   bash tools/gpu_quick2.sh OUTDIR
set -u
o=$1; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { echo tests failed; tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 240 python bench.py --no-e2e --no-cpu-baseline > $o/c2.json 2> $o/c2.err || { echo c2 failed; exit 1; }
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $o/c4.json 2> $o/c4.err || { echo c4 failed; exit 1; }
timeout -k 10 240 python bench.py --config c3 --no-cpu-baseline > $o/c3.json 2> $o/c3.err || { echo c3 failed; exit 1; }
timeout -k 10 300 python bench.py --config f3 > $o/f3.json 2> $o/f3.err || { echo f3 failed; exit 1; }
echo rc=0
