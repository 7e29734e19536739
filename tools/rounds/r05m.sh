#!/bin/bash
# r05m: the Tick hand-off defaults (sync: copy engine on a second stream, chunked; async: the same, chunked,
# two frames deep) -- rates at n = 1 and shared-device n = 2/8, then the whole GPU suite.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 300 python tools/tick_workers.py --configs C2,C3,C4,C5 --worlds 1 > $O/tick_n1.txt 2>&1 || { tail $O/tick_n1.txt; exit 1; }
cat $O/tick_n1.txt
timeout -k 10 300 python tools/tick_workers.py --configs C2,C5 --worlds 2,8 --shared > $O/tick_sh.txt 2>&1 || { tail $O/tick_sh.txt; exit 1; }
cat $O/tick_sh.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
