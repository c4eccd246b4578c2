#!/bin/bash
# N=2 rehearsal of bench.py's distributed path on a one-GPU box (two ranks share
# GPU 0 over gloo) + the C4 shard bench line.  Usage: bash tools/gpu_rehearse.sh OUTDIR
set -u
o=$1; mkdir -p $o
export PV_BENCH_BACKEND=gloo PV_BENCH_SHARE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $o/n2_c2.json 2> $o/n2_c2.err || { echo n2 failed; exit 1; }
unset PV_BENCH_BACKEND PV_BENCH_SHARE_GPU
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $o/c4.json 2> $o/c4.err || { echo c4 failed; exit 1; }
echo rc=0
