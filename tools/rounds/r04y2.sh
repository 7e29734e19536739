#!/bin/bash
# r04: the shadow grids with 16 and 64 axial slabs per light instead of 32 (whole-library builds,
# tools/build_full_variant.sh: lib/ab/libraytracer_hip_s16 / _s64) against the product: parity, then 64-frame
# launches of C4 / C5, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04y2
mkdir -p $O
L=$PWD/uu-infogr-raytracer_amd/lib
for v in s16 s64; do
    RAYTRACER_HIP_LIB=$L/ab/libraytracer_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
        -k "full_size or dense or bundle or shadow_grid or random" --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 \
        || { echo "PARITY FAILED $v"; tail -40 $O/parity_$v.log; exit 1; }
    echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2; do for c in C4 C5; do
    for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_s16.so $L/ab/libraytracer_hip_s64.so; do
        timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 256 --reps 3 --lib $lib \
            2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
    done
done; done
