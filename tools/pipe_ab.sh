set -e
o=gpurun_out/pipe_ab; mkdir -p $o
for rep in 1 2; do
for cfg in c2 c3; do
  timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --sequential > $o/${cfg}_seq_$rep.json 2>$o/${cfg}_seq_$rep.err
  timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $o/${cfg}_pipe_$rep.json 2>$o/${cfg}_pipe_$rep.err
done
done
echo done
