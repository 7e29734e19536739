#!/bin/bash
# r05c: which part of tests/test_gpu_tick.py leaves the process aborting at exit ("double free or corruption"
# after 80 passed, r05b): the RCCL-gather tests and the band-worker tests in processes of their own, with
# faulthandler's tracebacks on the abort.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 300 python -X faulthandler -u -m pytest tests/test_gpu_tick.py -k "not rccl" -x -q --timeout 120 --timeout-method thread > $O/workers.log 2>&1
echo "workers rc=$?"; tail -30 $O/workers.log
timeout -k 10 300 python -X faulthandler -u -m pytest tests/test_gpu_tick.py -k "rccl" -x -q --timeout 120 --timeout-method thread > $O/rccl.log 2>&1
echo "rccl rc=$?"; tail -30 $O/rccl.log
