set -u
o=gpurun_out/latx; mkdir -p $o
export PV_LAT_SIZES=1,1000,2048,4096,8192,16384,32768,65536,131072
timeout -k 10 200 python tools/latency.py > $o/default.jsonl 2> $o/default.err && \
PV_LAT_MAX=131072 timeout -k 10 200 python tools/latency.py > $o/lat131k.jsonl 2> $o/lat131k.err
echo rc=$?
