#!/bin/bash
# BLS GPU tests on the shipped (lane-pair) library, then an interleaved c3bls
# A/B against the one-lane variant, then the pair kernel's issue counters.
#   bash tools/gpu_bls_pair2.sh OUT
set -u
out=${1:-gpurun_out/bls_pair2}
mkdir -p "$out"
echo "[pair2] $(date +%T) tests" && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_bls_multi.py -x -q --timeout 300 --timeout-method thread -m gpu > "$out/tests.log" 2>&1 && \
echo "[pair2] $(date +%T) ab" && \
bash tools/ab_lib.sh "$out/ab" indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab/one_lane.so 2 --config c3bls --steps 3 --warmup 1 > "$out/ab.log" 2>&1 && \
echo "[pair2] $(date +%T) pmc" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_INT64 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$out/sq" -o pmc -- \
    python3 bench.py --config c3bls --steps 1 --warmup 0 --n 500000 --no-cpu-baseline > "$out/sq.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$out/lds" -o pmc -- \
    python3 bench.py --config c3bls --steps 1 --warmup 0 --n 500000 --no-cpu-baseline > "$out/lds.log" 2>&1 && \
echo "[pair2] done"
