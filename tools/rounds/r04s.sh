#!/bin/bash
# r04: lone frames of the bundle-kernel configs (C4, C5: one frame per rt_render_device launch) -- the product
# (natural order) and the bundle kernel with the lone-frame dispatch orders (profiles/ab/r04_bundle_lone_order.patch,
# lib/ab/libraytracer_hip_blo.so, RT_LONE_BUNDLE=1; measured choice and each order fixed) -- then the batch shape
# (64-frame launches) of both builds, and the parity suite of the variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04s
mkdir -p $O
L=uu-infogr-raytracer_amd/lib
BLO=$L/ab/libraytracer_hip_blo.so
RT_LONE_BUNDLE=1 RAYTRACER_HIP_LIB=$PWD/$BLO timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    -k "full_size or dense or bundle or shadow_grid or dispatch" --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 $O/parity.log; exit 1; }
echo "parity blo (RT_LONE_BUNDLE=1): $(tail -1 $O/parity.log)"
for rep in 1 2; do
    for c in C4 C5; do
        echo -n "[product] "
        timeout -k 10 180 python tools/frame_wall.py --config $c --batch 1 --frames 60 --reps 3 2>&1 | grep -v amdgpu.ids \
            | sed 's/strip=- bands=- //' || exit 1
        for o in auto 0 2; do
            echo -n "[blo order $o] "
            if [ $o = auto ]; then E=""; else E="RT_DISPATCH_ORDER=$o"; fi
            env RT_LONE_BUNDLE=1 $E timeout -k 10 180 python tools/frame_wall.py --config $c --batch 1 --frames 60 --reps 3 \
                --lib $BLO 2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
        done
        for lib in $L/libraytracer_hip.so $BLO; do
            timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 256 --reps 3 --lib $lib \
                2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
        done
    done
done
