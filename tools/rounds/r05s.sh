#!/bin/bash
# r05s: work-counter atomics spread over 8192 slots (product) against 256 (C256, the previous product) and none
# (NC, timing only) -- one-frame launches and 64-frame launches; then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05s
mkdir -p $O
BATCH=1 bash tools/ab_wall.sh "C2 C3 C4" lib/ab/libraytracer_hip_NC.so lib/ab/libraytracer_hip_C256.so lib/libraytracer_hip.so > $O/wall_b1.txt 2>&1 || { tail $O/wall_b1.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall_b1.txt
BATCH=64 bash tools/ab_wall.sh "C2 C3" lib/ab/libraytracer_hip_NC.so lib/ab/libraytracer_hip_C256.so lib/libraytracer_hip.so > $O/wall_b64.txt 2>&1 || { tail $O/wall_b64.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall_b64.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
