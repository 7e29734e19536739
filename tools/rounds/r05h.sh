#!/bin/bash
# r05h: kernel A/B -- base (round-start kernels), S (merged shadow loop without the per-light 2a check, light
# constants in two 16-byte scalar loads), product = S + the wave-uniform plane-division skip; then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05h
mkdir -p $O
bash tools/ab_wall.sh "C2 C3 C4 C5" lib/ab/libraytracer_hip_base.so lib/ab/libraytracer_hip_S.so lib/libraytracer_hip.so > $O/wall.txt 2>&1 || { tail $O/wall.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
