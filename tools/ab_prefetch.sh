set -u
o=gpurun_out/ab_pf; mkdir -p $o
timeout -k 10 300 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/libpv_nopf.so --rounds 6 > $o/c2.json 2> $o/c2.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
echo rc=$?
