#!/bin/bash
# r04: two tiles per workgroup for batch launches too (make variant NAME=w2all: RT_WPG_ALL=1 RT_SINGLE_WPG=2 --
# twice the tiles per dispatched workgroup, against the dispatcher's floor for one-wave groups) against the product:
# the batch-shape golden tests, 64-frame launches (C2, C3) and the driver's bench shape (C2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04t
mkdir -p $O
L=uu-infogr-raytracer_amd/lib
V=$PWD/$L/ab/libraytracer_hip_w2all.so
RAYTRACER_HIP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py -m gpu -x -q \
    -k "launch_shape or full_size or random_scenes or camera_sweep" --timeout 120 --timeout-method thread > $O/parity.log 2>&1 \
    || { echo "PARITY FAILED"; tail -40 $O/parity.log; exit 1; }
echo "parity w2all: $(tail -1 $O/parity.log)"
for rep in 1 2 3; do
    for c in C2 C3; do
        for lib in $PWD/$L/libraytracer_hip.so $V; do
            timeout -k 10 120 python tools/frame_wall.py --config $c --batch 64 --frames 1024 --reps 3 --lib $lib \
                2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
        done
    done
    for lib in $PWD/$L/libraytracer_hip.so $V; do
        RAYTRACER_HIP_LIB=$lib timeout -k 10 120 python bench.py --config C2 --steps 20 --warmup 5 --also "" --no-cpu-baseline \
            --no-tick > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$(basename $lib)', 'C2 driver shape', round(d['ms_per_step']*1e3, 3), 'us/frame')"
    done
done
# and the bundle kernel's shadow grids from fold level 2 instead of 1 (make variant NAME=g2 VFLAGS=-DRT_GRID_FROM_LEVEL=2)
G2=$PWD/$L/ab/libraytracer_hip_g2.so
if [ -f $G2 ]; then
    RAYTRACER_HIP_LIB=$G2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
        -k "full_size or dense or bundle or shadow_grid" --timeout 120 --timeout-method thread > $O/parity_g2.log 2>&1 \
        || { echo "PARITY FAILED g2"; tail -40 $O/parity_g2.log; exit 1; }
    echo "parity g2: $(tail -1 $O/parity_g2.log)"
    for rep in 1 2; do for c in C4 C5; do for lib in $PWD/$L/libraytracer_hip.so $G2; do
        timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 256 --reps 3 --lib $lib \
            2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
    done; done; done
fi
