#!/bin/bash
# round 3 batch C: k_keys with lane-interleaved scratch.  Keyed parity tests,
# C4 + C3 benches, rocprofv3 kernel stats of C4, k_keys FETCH/WRITE passes.
#   bash tools/gpu_r03_c.sh OUT
set -u
out=${1:-gpurun_out/r03_c}
mkdir -p "$out"
echo "[c] $(date +%T) tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_device.py tests/test_gpu_tally.py -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 && tail -1 "$out/tests.log" && \
echo "[c] $(date +%T) c4" && timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$out/c4.json" 2> "$out/c4.err" && \
echo "[c] $(date +%T) c3" && timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > "$out/c3.json" 2> "$out/c3.err" && \
echo "[c] $(date +%T) rocprof c4" && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_c4" -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --sequential --no-cpu-baseline --no-e2e > "$out/prof_c4.log" 2>&1 && \
echo "[c] $(date +%T) pmc" && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc/fetch" -o pmc -- python3 bench.py --config c4 --steps 1 --warmup 0 --n 2000000 --no-cpu-baseline --no-e2e > "$out/pmc_fetch.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc/write" -o pmc -- python3 bench.py --config c4 --steps 1 --warmup 0 --n 2000000 --no-cpu-baseline --no-e2e > "$out/pmc_write.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$out/pmc/sq" -o pmc -- python3 bench.py --config c4 --steps 1 --warmup 0 --n 2000000 --no-cpu-baseline --no-e2e > "$out/pmc_sq.log" 2>&1 && echo "[c] done"
