#!/bin/bash
# r04: single-frame dispatch orders (A/B through RT_ROW_ORDER: 0 natural, 1 rows by decreasing cost estimate,
# 2 reversed, 3 heaviest/lightest interleaved; RT_COL_MAJOR=1: rows vary fastest in dispatch order): parity of the
# column-major mapping, then wall per frame of back-to-back rt_render_device launches (C1, C2, C3).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04l
mkdir -p $O
RT_COL_MAJOR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/parity_cm.log 2>&1 || { echo "PARITY FAILED (col major)"; tail -40 $O/parity_cm.log; exit 1; }
echo "parity col-major: $(tail -1 $O/parity_cm.log)"
for rep in 1 2; do
    for c in C1 C2 C3; do
        for cm in 0 1; do
            for ro in 0 1 2 3; do
                echo -n "[RT_ROW_ORDER=$ro RT_COL_MAJOR=$cm] "
                RT_ROW_ORDER=$ro RT_COL_MAJOR=$cm timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 \
                    --frames 400 --reps 3 2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
            done
        done
    done
done
