#!/bin/bash
# r04: batch launches (64 frames) in the lone-frame dispatch orders (A/B, RT_BATCH_ORDER: 0 natural, 1 rows by
# estimated cost, 2 rows bottom to top, 3 rows varying fastest): the batch-shape golden tests under 2 and 3, then
# wall per frame, C2 / C3, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04n
mkdir -p $O
for bo in 2 3; do
    RT_BATCH_ORDER=$bo timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q -k "launch_shape or count_work" \
        --timeout 120 --timeout-method thread > $O/parity_$bo.log 2>&1 || { echo "PARITY FAILED $bo"; tail -40 $O/parity_$bo.log; exit 1; }
    echo "parity RT_BATCH_ORDER=$bo: $(tail -1 $O/parity_$bo.log)"
done
for rep in 1 2; do
    for c in C2 C3; do
        for bo in 0 1 2 3; do
            echo -n "[RT_BATCH_ORDER=$bo] "
            RT_BATCH_ORDER=$bo timeout -k 10 120 python tools/frame_wall.py --config $c --batch 64 --frames 1024 --reps 3 \
                2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
        done
    done
done
