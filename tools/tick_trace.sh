#!/bin/bash
# Tick() hand-off probe, plain and under a kernel + memory-copy + HIP-runtime trace (no counters).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/tick_trace

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d $R/gpurun_out/tick_trace/prof -o tick -- python3 -u $R/tools/tick_trace.py > $R/gpurun_out/tick_trace/traced.txt 2>&1
