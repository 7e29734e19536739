#!/bin/bash
# r04: single-frame launches with the tile rows sorted by the host's cost estimate (LaunchParams::row_order)
# against the natural order (RT_ROW_ORDER=0): GPU parity, wall per frame (C2 / C3 / empty C2, alternating), then the
# wave timelines of both orders (probe build) with per-tile durations saved for offline ordering studies.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
for rep in 1 2; do
    for c in "C2" "C3" "C1" "C2 --strip spheres,planes,lights"; do
        for ro in 0 1; do
            echo -n "[RT_ROW_ORDER=$ro] "
            RT_ROW_ORDER=$ro timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 \
                2>&1 | grep -v amdgpu.ids | sed 's/bands=- //' || exit 1
        done
    done
done
WT=uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_wt.so
for c in C2 C3; do
    for ro in 1 0; do
        echo "== $c single frame, RT_ROW_ORDER=$ro"
        RT_ROW_ORDER=$ro timeout -k 10 120 python tools/wave_times.py --lib $WT --config $c --batch 1 \
            --save $O/wt_${c}_ro$ro.npz 2>&1 | grep -v amdgpu.ids | grep -v "^   (" || exit 1
    done
done
