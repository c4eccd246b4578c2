#!/bin/bash
# Round 6: sigma's prep on a lane pair in k_bls_prep (one root/inverse-root
# exponentiation instead of a root then an inversion).  BLS GPU tests, then
# lone-check / 3PC-batch latencies interleaved against -D PV_SIGPREP_PAIR=0
# (indy-plenum_amd/lib/ab_sigprep_one.so), three rounds, and a kernel trace.
# Not adopted: the variant is tools/ab/bls_sigprep_pair_notadopted.patch (apply it
# and add the PV_SIGPREP_PAIR switch to rebuild the A/B pair).
#   bash tools/gpu_bls_siglat.sh OUT
set -u
out=${1:-gpurun_out/siglat}
mkdir -p "$out"
echo "[sl] $(date +%T) tests" && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bls.py tests/test_gpu_bls_multi.py > "$out/tests.log" 2>&1 && \
for r in 1 2 3; do
  for lib in indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/ab_sigprep_one.so; do
    tag=$(basename $lib .so)
    echo "[sl] $(date +%T) $tag $r"
    PLENUM_GPU_LIB=$lib timeout -k 10 120 python tools/bls_latency.py 1 25 250 > "$out/lat_${tag}_$r.jsonl" 2>/dev/null || exit 1
  done
done && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 tools/bls_latency.py 1 25 > "$out/prof.log" 2>&1 && \
echo "[sl] done"
