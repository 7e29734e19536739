#!/bin/bash
# A/B of rt_render_async's hand-off (RT_ASYNC_MODE: 0 two streams + events, 1 one stream, 2 zero-copy), no profiler.
# (historical: RT_ASYNC_MODE was removed from rt_api.cpp after this A/B; profiles/r03_tick_ab.txt holds its output)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/tick_ab
for m in 0 1 2 0 1 2; do
  echo "== RT_ASYNC_MODE=$m" >> $R/gpurun_out/tick_ab/ab.txt
  RT_ASYNC_MODE=$m timeout -k 10 120 python3 -u $R/tools/tick_trace.py >> $R/gpurun_out/tick_ab/ab.txt 2>&1
done
