#!/bin/bash
# r05r: the lone frame's extra cost -- product vs NC (tools/ablate/r05_nocount.patch: no work-counter atomics)
# for one-frame launches (BATCH=1, what Tick / single_launch_fps issue) and the bench's 64-frame launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05r
mkdir -p $O
BATCH=1 bash tools/ab_wall.sh "C2 C3 C4" lib/ab/libraytracer_hip_NC.so lib/libraytracer_hip.so > $O/wall_b1.txt 2>&1 || { tail $O/wall_b1.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall_b1.txt
BATCH=64 bash tools/ab_wall.sh "C3 C4" lib/ab/libraytracer_hip_NC.so lib/libraytracer_hip.so > $O/wall_b64.txt 2>&1 || { tail $O/wall_b64.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall_b64.txt
