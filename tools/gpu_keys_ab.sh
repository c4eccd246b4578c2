#!/bin/bash
# k_keys at 2 (default) vs 3 waves/SIMD (variant lib, -DPV_KEYS_WAVES=3): C4
# bench lines interleaved, plus the keyed GPU tests on the variant.
#   bash tools/gpu_keys_ab.sh OUT
set -u
out=${1:-gpurun_out/keys_ab}
mkdir -p "$out"
PLENUM_GPU_LIB=$PWD/indy-plenum_amd/lib/var_keys3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -q \
  --timeout 200 --timeout-method thread -k "keyed or prepared or dedup" > "$out/tests_var.log" 2>&1 || { tail -20 "$out/tests_var.log"; exit 1; }
grep passed "$out/tests_var.log"
for k in 1 2; do
  for v in default var; do
    if [ $v = var ]; then export PLENUM_GPU_LIB=$PWD/indy-plenum_amd/lib/var_keys3.so; else unset PLENUM_GPU_LIB; fi
    timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > "$out/c4_$v.$k.json" 2> "$out/c4_$v.$k.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['kernel_ms'], d['verdict_mismatches'])" "$out/c4_$v.$k.json"
  done
done
