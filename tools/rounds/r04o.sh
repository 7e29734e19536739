#!/bin/bash
# r04: software-pipelined candidate loops -- the next candidate's sphere record loads while the current one is tested:
# the merged shadow loop (profiles/ab/r04_merged_prefetch.patch, pfm), the trace bundles' pair loop (profiles/ab/r04_walk_prefetch.patch,
# pfw), both (profiles/ab/r04_prefetch_both.patch, pfb) -- against the product build: parity, then
# wall per frame of 64-frame launches, C4 / C5, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04o
mkdir -p $O
L=uu-infogr-raytracer_amd/lib
for v in pfm pfw pfb; do
    RAYTRACER_HIP_LIB="$PWD/$L/ab/libraytracer_hip_$v.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
        --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || { echo "PARITY FAILED $v"; tail -40 $O/parity_$v.log; exit 1; }
    echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2; do
    for c in C4 C5; do
        for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_pfm.so $L/ab/libraytracer_hip_pfw.so $L/ab/libraytracer_hip_pfb.so; do
            timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 512 --reps 3 --lib $lib \
                2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
        done
    done
done
