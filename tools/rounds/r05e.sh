#!/bin/bash
# r05e: the synchronous Tick's hand-off, copy engine (pitched copies into the registered frame) against the
# copy kernel (chunked), at n = 1 and with n workers sharing the one device (one PCIe link).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05e
mkdir -p $O
for c in runtime kernel; do
  timeout -k 10 300 python tools/tick_workers.py --configs C2,C5 --worlds 2,4,8 --shared --copy $c --chunks 1,2 > $O/tick_$c.txt 2>&1 || { tail $O/tick_$c.txt; exit 1; }
  cat $O/tick_$c.txt
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_tick.py -x -q --timeout 120 --timeout-method thread > $O/tick_tests.log 2>&1; echo "tick tests rc=$? $(tail -1 $O/tick_tests.log)"
RT_TICK_COPY=runtime timeout -k 10 300 python -u -m pytest tests/test_gpu_tick.py -x -q --timeout 120 --timeout-method thread > $O/tick_tests_rt.log 2>&1; echo "tick tests (runtime copies) rc=$? $(tail -1 $O/tick_tests_rt.log)"
