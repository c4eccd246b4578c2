#!/bin/bash
# Round-6 closing evidence on the current build: the -m gpu suite and smoke(),
# the default bench line (C2 + every other config), rocprofv3 kernel stats of
# the C2 / C4 / C3 lines run sequentially (the roofline's kernel durations) and of the
# C3-BLS line.  Each GPU step under its own limit; the chain stops at a failure.
#   bash tools/gpu_r06_final.sh OUT
set -u
out=${1:-gpurun_out/r06final}
mkdir -p "$out"
# a rocprofv3 database -> kernel table (tools/rocpd_stats.py); the raw output is
# removed so gpurun_out stays under the 64 MiB copy-back limit
stats() {
  db=$(find "$out/$1" -name '*.db' -print -quit)
  [ -n "$db" ] && python3 tools/rocpd_stats.py "$db" > "$out/$1_kernel_stats.txt" && rm -rf "$out/$1"
}
echo "[final] $(date +%T) suite" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1 && \
echo "[final] $(date +%T) smoke" && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 && \
echo "[final] $(date +%T) bench" && \
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
echo "[final] $(date +%T) stats c2" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/c2_seq" -o run -- python3 bench.py --sequential \
    --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-other-configs > "$out/c2_seq.json" 2> "$out/c2_seq.err" && \
stats c2_seq && \
echo "[final] $(date +%T) stats c4" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c4_seq" -o run -- python3 bench.py --config c4 --sequential \
    --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$out/c4_seq.json" 2> "$out/c4_seq.err" && \
stats c4_seq && \
echo "[final] $(date +%T) stats c3" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c3_seq" -o run -- python3 bench.py --config c3 --sequential \
    --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > "$out/c3_seq.json" 2> "$out/c3_seq.err" && \
stats c3_seq && \
echo "[final] $(date +%T) stats c3bls" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c3bls" -o run -- python3 bench.py --config c3bls \
    --steps 3 --warmup 1 --no-cpu-baseline > "$out/c3bls.json" 2> "$out/c3bls.err" && \
stats c3bls && echo "[final] done"
