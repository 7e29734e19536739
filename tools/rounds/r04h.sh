#!/bin/bash
# r04: wave timelines of single-frame and batched direct-kernel launches (tools/wave_times.py on the probe build
# lib/ab/libraytracer_hip_wt.so, tools/build_wave_times.sh), C2 and C3; single frames in the host's row order
# (default) and in the natural one (RT_ROW_ORDER=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
WT=uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_wt.so
for c in C2 C3; do
    echo "== $c single frame, host row order"
    timeout -k 10 120 python tools/wave_times.py --lib $WT --config $c --batch 1 --map 2>&1 | grep -v amdgpu.ids || exit 1
    echo "== $c single frame, natural row order"
    RT_ROW_ORDER=0 timeout -k 10 120 python tools/wave_times.py --lib $WT --config $c --batch 1 2>&1 | grep -v amdgpu.ids || exit 1
    echo "== $c 4-frame launch"
    timeout -k 10 120 python tools/wave_times.py --lib $WT --config $c --batch 4 2>&1 | grep -v amdgpu.ids || exit 1
    timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 --lib $WT 2>&1 | grep -v amdgpu.ids || exit 1
done
