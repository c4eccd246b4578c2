mkdir -p gpurun_out/ab4
timeout -k 10 300 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/libpv_words.so --rounds 5 > gpurun_out/ab4/c2.json 2> gpurun_out/ab4/c2.err && \
timeout -k 10 300 python tools/variant_bench.py indy-plenum_amd/lib/libplenum_verify.so indy-plenum_amd/lib/libpv_words.so --rounds 3 --n 2000000 --mode 1 --mlen 128 --mlen-max 4096 --cfg 4 > gpurun_out/ab4/c4.json 2> gpurun_out/ab4/c4.err
