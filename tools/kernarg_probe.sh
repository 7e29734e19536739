#!/bin/bash
# Does the kernarg placement matter?  Wall per frame (bench shape) with the runtime's default
# kernarg placement vs HIP_FORCE_DEV_KERNARG=1, full scene and empty scene.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in C2 C3; do
  for s in "" "spheres,planes,lights"; do
    for env in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0"; do
      echo -n "[$env] "
      env $env timeout -k 10 120 python tools/frame_wall.py --config $c --inflight 1 --batch 64 --frames 1024 \
        ${s:+--strip $s} 2>&1 | grep -v amdgpu.ids || exit $?
    done
  done
done
