#!/bin/bash
# One GPU session: full -m gpu suite, every bench config, rocprofv3 kernel
# stats of the headline bench (pipelined default AND --sequential, whose
# per-launch durations are the ones bench.py's kernel events measure), the
# latency sweep and the PMC passes.  Run on the GPU box:
#   bash tools/gpu_round.sh gpurun_out/round
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
out=${1:-gpurun_out/round}
mkdir -p "$out"
step() { echo "[gpu_round] $(date +%T) $1" | tee -a "$out/steps.log"; }
step tests && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 && tail -1 "$out/gpu_tests.log" && \
step c2 && timeout -k 10 300 python bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err" && \
step c1 && timeout -k 10 240 python bench.py --config c1 > "$out/bench_c1.json" 2> "$out/bench_c1.err" && \
step c3 && timeout -k 10 240 python bench.py --config c3 > "$out/bench_c3.json" 2> "$out/bench_c3.err" && \
step c4 && timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 > "$out/bench_c4.json" 2> "$out/bench_c4.err" && \
step f3 && timeout -k 10 240 python bench.py --config f3 > "$out/bench_f3.json" 2> "$out/bench_f3.err" && \
step latency && timeout -k 10 240 python tools/latency.py > "$out/latency.jsonl" 2> "$out/latency.err" && \
step rocprof && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --no-cpu-baseline --no-e2e \
    > "$out/prof.log" 2>&1 && \
step rocprof_seq && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_seq" -o run -- python3 bench.py \
    --sequential --no-cpu-baseline --no-e2e > "$out/prof_seq.log" 2>&1 && \
step pmc && bash tools/pmc_passes.sh "$out/pmc" && step done
