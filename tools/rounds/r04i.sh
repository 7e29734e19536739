#!/bin/bash
# r04: single-frame launches with the tile rows in the host's cost order (LaunchParams::row_rev, expensive rows
# first) against the natural order (RT_ROW_ORDER=0): GPU parity suite, then wall per frame of back-to-back
# rt_render_device launches, C2 / C3 / the empty C2 scene, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
for rep in 1 2; do
    for c in "C2" "C3" "C2 --strip spheres,planes,lights"; do
        for ro in 0 1; do
            echo -n "[RT_ROW_ORDER=$ro] "
            RT_ROW_ORDER=$ro timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 \
                2>&1 | grep -v amdgpu.ids | sed 's/bands=- //' || exit 1
        done
    done
done
