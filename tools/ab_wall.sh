#!/bin/bash
# A/B of library builds by wall time per frame (tools/frame_wall.py: the bench's shape, 64 frames
# per launch, one launch in flight), alternating builds, two passes per config.  Usage (GPU box):
#   bash tools/ab_wall.sh "C2 C3 C4" lib/ab/libraytracer_hip_X.so lib/libraytracer_hip.so ...
# EXTRA="--strip spheres" etc. is passed to frame_wall.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfgs=$1; shift
for c in $cfgs; do
    for rep in 1 2; do
        for lib in "$@"; do
            timeout -k 10 180 python tools/frame_wall.py --config "$c" --inflight ${INFLIGHT:-1} --batch ${BATCH:-64} --frames 1024 \
                --lib "uu-infogr-raytracer_amd/$lib" ${EXTRA:-} 2>&1 | grep -v amdgpu.ids || exit $?
        done
    done
done
