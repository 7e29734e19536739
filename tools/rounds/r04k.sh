#!/bin/bash
# r04: issue priority for long mirror chains (profiles/ab/r04_tail_prio.patch: s_setprio 2 once a wave's lanes reach 1 / 2
# reflections; lib/ab/libraytracer_hip_tp1 / _tp2) against the product build: parity, single-frame wall (C2, C3),
# and the batch shape (64-frame launches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04k
mkdir -p $O
L=uu-infogr-raytracer_amd/lib
for v in tp1 tp2; do
    RAYTRACER_HIP_LIB="$PWD/$L/ab/libraytracer_hip_$v.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
        --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || { echo "PARITY FAILED $v"; tail -40 $O/parity_$v.log; exit 1; }
    echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2; do
    for c in C2 C3; do
        for ro in 0 1; do
            for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_tp1.so $L/ab/libraytracer_hip_tp2.so; do
                echo -n "[RT_ROW_ORDER=$ro] "
                RT_ROW_ORDER=$ro timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 --lib $lib \
                    2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
            done
        done
    done
done
for c in C2 C3; do
    for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_tp1.so $L/ab/libraytracer_hip_tp2.so; do
        timeout -k 10 120 python tools/frame_wall.py --config $c --batch 64 --frames 1024 --lib $lib \
            2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
    done
done
