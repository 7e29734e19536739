#!/bin/bash
# r04: lone frames of the bundle-kernel configs (C4, C5: one frame per rt_render_device launch) against their
# 64-frame launches -- the size of the lone-frame tail on the bundle kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for rep in 1 2; do
    for c in C4 C5; do
        for b in 1 64; do
            timeout -k 10 180 python tools/frame_wall.py --config $c --batch $b --frames $((b == 1 ? 200 : 256)) --reps 3 \
                2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
        done
    done
done
