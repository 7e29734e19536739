#!/bin/bash
# r04: trace bundles that allow no culling take every sphere without the per-lane cull arithmetic
# (profiles/ab/r04_nocull.patch: ncA when the bound is unusable, ncB also when its cone is wider than 0.25) against the
# product: parity, then 64-frame launches of C4 / C5, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04y3
mkdir -p $O
L=$PWD/uu-infogr-raytracer_amd/lib
for v in ncA ncB; do
    RAYTRACER_HIP_LIB=$L/ab/libraytracer_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
        -k "full_size or dense or bundle or shadow_grid or random" --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 \
        || { echo "PARITY FAILED $v"; tail -40 $O/parity_$v.log; exit 1; }
    echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2; do for c in C4 C5; do
    for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_ncA.so $L/ab/libraytracer_hip_ncB.so; do
        timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 256 --reps 3 --lib $lib \
            2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
    done
done; done
