#!/bin/bash
# Where the C2 frame time goes: wall per frame at the bench's shape with parts of the scene removed
# (tools/frame_wall.py --strip), in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in "" lights spheres planes "spheres,planes,lights"; do
    timeout -k 10 120 python tools/frame_wall.py --config ${CFG:-C2} --inflight 1 --batch 64 --frames 1024 \
        ${s:+--strip $s} 2>&1 | grep -v amdgpu.ids || exit $?
done
