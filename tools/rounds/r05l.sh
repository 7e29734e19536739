#!/bin/bash
# r05l: rt_render_async's hand-off by the copy engine on a second stream (RT_TICK_ASYNC=stream) against the
# copy slice in the next launch, and the synchronous Tick's new default (stream, chunked); Tick tests under both.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05l
mkdir -p $O
for a in slice stream; do
  timeout -k 10 300 python tools/tick_workers.py --configs C2,C3,C4,C5 --worlds 1 --async-copy $a > $O/tick_n1_$a.txt 2>&1 || { tail $O/tick_n1_$a.txt; exit 1; }
  cat $O/tick_n1_$a.txt
  timeout -k 10 300 python tools/tick_workers.py --configs C2,C5 --worlds 2,8 --shared --async-copy $a > $O/tick_sh_$a.txt 2>&1 || { tail $O/tick_sh_$a.txt; exit 1; }
  cat $O/tick_sh_$a.txt
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_tick.py -x -q --timeout 120 --timeout-method thread > $O/tick_tests.log 2>&1; echo "tick tests rc=$? $(tail -1 $O/tick_tests.log)"
RT_TICK_ASYNC=stream timeout -k 10 300 python -u -m pytest tests/test_gpu_tick.py tests/test_gpu_parity.py -k "tick or async" -x -q --timeout 120 --timeout-method thread > $O/tick_tests_as.log 2>&1; echo "tick+async tests (async stream) rc=$? $(tail -1 $O/tick_tests_as.log)"
