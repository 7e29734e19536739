#!/bin/bash
# r04 third GPU call: the merged-pass instantiation (MERGED) with the shadow grids from fold level 1
# (mg1: level 0 keeps the per-level bound) or 0 (mg0: grids everywhere) against r03 (base) and the
# first grid build (nopk); mg1 with RT_SHADOW_GRID=0 is MERGED with the bound alone.  Then the
# N > 1 default path's stage table without the post-run verification.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04c
mkdir -p $O
B=lib/ab/libraytracer_hip_base.so
N=lib/ab/libraytracer_hip_nopk.so
M0=lib/ab/libraytracer_hip_mg0.so
M1=lib/ab/libraytracer_hip_mg1.so
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$M1" timeout -k 10 500 python -u -m pytest tests -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity_mg1.log 2>&1 || { echo "PARITY FAILED $M1"; tail -40 $O/parity_mg1.log; exit 1; }
echo "parity (whole GPU suite) $M1: $(tail -1 $O/parity_mg1.log)"
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$M0" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity_mg0.log 2>&1 || { echo "PARITY FAILED $M0"; tail -40 $O/parity_mg0.log; exit 1; }
echo "parity $M0: $(tail -1 $O/parity_mg0.log)"
for c in C4 C5; do
    for rep in 1 2; do
        for lib in $B $N $M0 $M1; do
            timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 1024 --lib uu-infogr-raytracer_amd/$lib \
                2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
        done
        echo -n "[RT_SHADOW_GRID=0] "
        RT_SHADOW_GRID=0 timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 1024 \
            --lib uu-infogr-raytracer_amd/$M1 2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
    done
done
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"
bash tools/pmc_ab.sh C4 "$PMC" $B $M1 || exit 1
DIST_FLAGS="--no-verify" DIST_OUT=r04_dist_direct bash tools/dist_trace.sh || exit 1
head -40 gpurun_out/r04_dist_direct/stages.txt
