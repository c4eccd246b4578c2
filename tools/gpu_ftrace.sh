set -u
o=gpurun_out/ftrace; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $o/trace -- python3 tools/e2e_trace.py > $o/trace.log 2>&1 || { echo trace failed; tail $o/trace.log; exit 1; }
echo ok
