#!/bin/bash
# r04: the bundle kernel at 96 SGPRs / 7 waves per SIMD (profiles/ab/r04_sgpr96.patch: no SGPR spills in the merged
# instantiation) against the product's 80 SGPRs / 8 waves (11 SGPRs spilled to VGPR lanes): parity, then wall per
# frame of 64-frame launches, C4 / C5, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04r
mkdir -p $O
L=uu-infogr-raytracer_amd/lib
RAYTRACER_HIP_LIB="$PWD/$L/ab/libraytracer_hip_s96.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 $O/parity.log; exit 1; }
echo "parity s96: $(tail -1 $O/parity.log)"
for rep in 1 2; do
    for c in C4 C5; do
        for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_s96.so; do
            timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 512 --reps 3 --lib $lib \
                2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
        done
    done
done
