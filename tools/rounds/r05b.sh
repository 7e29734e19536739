#!/bin/bash
# r05b: the ABI 9 multi-GPU Tick (per-worker PCIe hand-off, chunked synchronous copies, double-buffered
# workers) -- its GPU tests, the whole GPU suite, then Tick rates by chunk count at n = 1 and the
# shared-device workers (one link: a code-path check, not a scaling number).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -X faulthandler -u -m pytest tests/test_gpu_tick.py -x -q --timeout 120 --timeout-method thread > $O/tick_tests.log 2>&1 \
    || { echo "TICK TESTS FAILED"; tail -40 $O/tick_tests.log; exit 1; }
echo "tick tests: $(tail -1 $O/tick_tests.log)"
timeout -k 10 600 python -X faulthandler -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -40 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
timeout -k 10 300 python tools/tick_workers.py --configs C2,C3,C4,C5 --worlds 1 --chunks 1,2,4,8 > $O/tick_n1.txt 2>&1 || { tail $O/tick_n1.txt; exit 1; }
cat $O/tick_n1.txt
timeout -k 10 300 python tools/tick_workers.py --configs C2,C5 --worlds 2,4,8 --shared > $O/tick_shared.txt 2>&1 || { tail $O/tick_shared.txt; exit 1; }
cat $O/tick_shared.txt
