#!/bin/bash
# Round 3: the fused Tick hand-off -- its GPU tests first, then the whole GPU suite, the hand-off probe
# (fused vs RT_ASYNC_NOFUSE, i.e. one stream with the runtime's copy) and the default bench line.
# (historical: RT_ASYNC_NOFUSE was removed after this A/B; profiles/r03_tick_ab.txt holds its output)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03a
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "async" > $O/pytest_async.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -u tools/tick_trace.py > $O/tick_fused.txt 2>&1
RT_ASYNC_NOFUSE=1 timeout -k 10 120 python3 -u tools/tick_trace.py > $O/tick_nofuse.txt 2>&1
timeout -k 10 120 python3 -u tools/tick_trace.py > $O/tick_fused2.txt 2>&1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
# the N > 1 pipeline in one process (RCCL world of 1): C2, then C5 through the also-dist leg
timeout -k 10 300 python3 -u bench.py --dist-path --rank0-codec --steps 20 --warmup 5 --verify > $O/distpath.json 2> $O/distpath.err
