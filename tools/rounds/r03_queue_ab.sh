#!/bin/bash
# A/B of the shadow queue (in-tree, RT_SHADOW_QUEUE=1) against the merged per-level shadow pass
# (lib/ab/libraytracer_hip_noqueue.so): GPU parity suite of the in-tree build, wall per frame C4/C5,
# lane-slot utilisation (slot variants built with the queue).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_wall.sh "C4 C5" lib/libraytracer_hip.so lib/ab/libraytracer_hip_noqueue.so > $O/wall.txt 2>&1 || exit 1
cat $O/wall.txt
timeout -k 10 600 python3 -u tools/slot_probe.py --configs C4 C5 > $O/slot_probe.txt 2>&1 || exit 1
cat $O/slot_probe.txt
