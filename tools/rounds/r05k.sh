#!/bin/bash
# r05k: the synchronous Tick's chunked copy-engine hand-off on a second stream (RT_TICK_COPY=stream) against
# the runtime copy after the trace (n = 1 default) and the copy kernel; then the Tick tests in stream mode.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05k
mkdir -p $O
for c in runtime stream; do
  timeout -k 10 300 python tools/tick_workers.py --configs C2,C3,C4,C5 --worlds 1 --copy $c --chunks 1,2,4,8 > $O/tick_n1_$c.txt 2>&1 || { tail $O/tick_n1_$c.txt; exit 1; }
  cat $O/tick_n1_$c.txt
done
for c in kernel stream; do
  timeout -k 10 300 python tools/tick_workers.py --configs C2,C5 --worlds 2,8 --shared --copy $c > $O/tick_sh_$c.txt 2>&1 || { tail $O/tick_sh_$c.txt; exit 1; }
  cat $O/tick_sh_$c.txt
done
RT_TICK_COPY=stream timeout -k 10 300 python -u -m pytest tests/test_gpu_tick.py -x -q --timeout 120 --timeout-method thread > $O/tick_tests_stream.log 2>&1; echo "tick tests (stream) rc=$? $(tail -1 $O/tick_tests_stream.log)"
