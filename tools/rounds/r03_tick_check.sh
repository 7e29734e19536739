#!/bin/bash
# The fused Tick hand-off: its GPU tests, the hand-off probe and the bench's Tick rates (C2).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03t
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "async" > $O/pytest_async.log 2>&1
timeout -k 10 120 python3 -u tools/tick_trace.py > $O/tick_fused.txt 2>&1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --also "" > $O/bench.json 2> $O/bench.err
