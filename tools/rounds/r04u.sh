#!/bin/bash
# r04: at the first fold level, the ball bound when the wave's hit points lie within K grid cells of their centre and
# the shadow grid otherwise (profiles/ab/r04_adapt_level1.patch, K = 1 / 2 / 4: lib/ab/libraytracer_hip_ad1/2/4) against the
# product (grid at every level >= 1): parity, then 64-frame launches of C4 / C5, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04u
mkdir -p $O
L=$PWD/uu-infogr-raytracer_amd/lib
for v in ad1 ad4; do
    RAYTRACER_HIP_LIB=$L/ab/libraytracer_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
        -k "full_size or dense or bundle or shadow_grid or random" --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 \
        || { echo "PARITY FAILED $v"; tail -40 $O/parity_$v.log; exit 1; }
    echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2; do for c in C4 C5; do
    for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_ad1.so $L/ab/libraytracer_hip_ad2.so $L/ab/libraytracer_hip_ad4.so; do
        timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 256 --reps 3 --lib $lib \
            2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
    done
done; done
