#!/bin/bash
# Host-buffer pipeline check: -m gpu suite, the c2 bench line with end_to_end,
# and a rocprofv3 kernel timeline of the host-buffer call.  bash tools/gpu_e2e.sh OUTDIR
set -u
o=$1; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { echo tests failed; tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $o/c2.json 2> $o/c2.err || { echo c2 failed; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $o/trace -- python3 tools/e2e_trace.py > $o/trace.log 2>&1 || { echo trace failed; exit 1; }
echo rc=0
