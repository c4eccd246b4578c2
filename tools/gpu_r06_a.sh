#!/bin/bash
# Round 6, first GPU pass: the touched GPU tests (key cache / completion word,
# BLS shutdown cycle, RCCL + bench self-launch), the int-rate micro-benchmark
# (v_bitop3 / v_lshrrev_b32 / v_perm for the k_hash roofline), C4 + C2 lines
# with the hash roofline and stage sums.  Each GPU step under its own limit.
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06a
O=gpurun_out/r06a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_keycache.py \
  tests/test_gpu_bls.py tests/test_gpu_rccl.py > $O/tests.log 2>&1
echo tests ok
timeout -k 10 60 tools/ubench/int_rates > $O/int_rates.json
echo rates ok
timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err
echo c4 ok
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 2 --no-other-configs --no-e2e > $O/c2.json 2> $O/c2.err
echo c2 ok
