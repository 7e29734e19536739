#!/bin/bash
# GPU box: launches in flight (1/2/3) x frames per launch (1/16), C2 and C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in C2 C4; do for b in 16 32; do for i in 1 2 3; do
  timeout -k 10 120 python tools/frame_wall.py --config $c --inflight $i --batch $b --frames 640 2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //'
done; done; done
