#!/bin/bash
# End-of-session GPU round: smoke(), the -m gpu suite, every bench config, the
# latency sweep, rocprofv3 kernel stats (pipelined + sequential C2).
#   bash tools/gpu_final.sh OUT
set -u
out=${1:-gpurun_out/final}
mkdir -p "$out"
step() { echo "[gpu_final] $(date +%T) $1" | tee -a "$out/steps.log"; }
step smoke && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 && tail -1 "$out/smoke.log" && \
step tests && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 && tail -1 "$out/gpu_tests.log" && \
step c2 && timeout -k 10 300 python bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err" && \
step c1 && timeout -k 10 240 python bench.py --config c1 > "$out/bench_c1.json" 2> "$out/bench_c1.err" && \
step c3 && timeout -k 10 240 python bench.py --config c3 > "$out/bench_c3.json" 2> "$out/bench_c3.err" && \
step c4 && timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 > "$out/bench_c4.json" 2> "$out/bench_c4.err" && \
step f3 && timeout -k 10 240 python bench.py --config f3 > "$out/bench_f3.json" 2> "$out/bench_f3.err" && \
step c3bls && timeout -k 10 300 python bench.py --config c3bls > "$out/bench_c3bls.json" 2> "$out/bench_c3bls.err" && \
step latency && timeout -k 10 240 python tools/latency.py > "$out/latency.jsonl" 2> "$out/latency.err" && \
PV_LAT_CACHED=1 timeout -k 10 240 python tools/latency.py > "$out/latency_cached.jsonl" 2>> "$out/latency.err" && \
step rocprof && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --no-cpu-baseline --no-e2e \
    > "$out/prof.log" 2>&1 && \
step rocprof_seq && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_seq" -o run -- python3 bench.py \
    --sequential --no-cpu-baseline --no-e2e > "$out/prof_seq.log" 2>&1 && step done
