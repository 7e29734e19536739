#!/bin/bash
# r05f: the copy kernel's host writes with the frame locked coarse-grained (RT_HOST_REGISTER=coarse) against
# the default fine-grained lock: Tick rates (copy kernel, chunked; copy slices in the async path) and the
# Tick tests under it (every frame = golden / oracle, guards intact).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05f
mkdir -p $O
for reg in fine coarse; do
  RT_HOST_REGISTER=$reg timeout -k 10 300 python tools/tick_workers.py --configs C2,C5 --worlds 1 --copy kernel --chunks 1,2,4 > $O/tick_n1_$reg.txt 2>&1 || { tail $O/tick_n1_$reg.txt; exit 1; }
  sed "s/^/$reg /" $O/tick_n1_$reg.txt
  RT_HOST_REGISTER=$reg timeout -k 10 300 python tools/tick_workers.py --configs C2,C5 --worlds 4,8 --shared --copy kernel --chunks 1,2 > $O/tick_sh_$reg.txt 2>&1 || { tail $O/tick_sh_$reg.txt; exit 1; }
  sed "s/^/$reg /" $O/tick_sh_$reg.txt
done
RT_HOST_REGISTER=coarse timeout -k 10 300 python -u -m pytest tests/test_gpu_tick.py -x -q --timeout 120 --timeout-method thread > $O/tick_tests_coarse.log 2>&1; echo "tick tests (coarse) rc=$? $(tail -1 $O/tick_tests_coarse.log)"
