#!/bin/bash
# smoke() + N=2 rehearsal of the multi-rank bench loop on one GPU (gloo
# collectives through host copies, both ranks on GPU 0).  Run on the GPU box:
#   bash tools/gpu_check.sh gpurun_out/check
set -u
out=${1:-gpurun_out/check}
mkdir -p "$out"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 && \
PV_BENCH_BACKEND=gloo PV_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 \
  --no-cpu-baseline > "$out/rehearsal_n2_c2.json" 2> "$out/rehearsal_n2_c2.err"
echo "rc=$?"
