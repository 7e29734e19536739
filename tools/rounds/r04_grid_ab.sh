#!/bin/bash
# r04 A/B: per-light shadow grids (lib/ab/libraytracer_hip_grid.so) against the per-level bound
# (lib/ab/libraytracer_hip_base.so = the build before them), and the direct kernel's packed sphere
# pairs (libraytracer_hip_pk.so = grid + packed; _nopk = grid + the scalar direct loops): the whole
# GPU suite on the grid and packed builds, wall per frame C4/C5 and C2/C3 alternating, PMC
# instruction mix per dispatch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04g
mkdir -p $O
B=lib/ab/libraytracer_hip_base.so
G=lib/ab/libraytracer_hip_nopk.so  # grid, scalar direct loops
P=lib/ab/libraytracer_hip_pk.so
N=$G
T=lib/ab/libraytracer_hip_pkth.so  # packed + the division-free shadow threshold in the direct kernel
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$G" timeout -k 10 500 python -u -m pytest tests -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity_grid.log 2>&1 || { echo "PARITY FAILED $G"; tail -40 $O/parity_grid.log; exit 1; }
echo "parity (whole GPU suite) $G: $(tail -1 $O/parity_grid.log)"
for lib in $P $T; do  # the direct kernel's variants: the parity suite proper
    RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$lib" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu \
        -x -q --timeout 120 --timeout-method thread > $O/parity_$(basename $lib .so).log 2>&1 \
        || { echo "PARITY FAILED $lib"; tail -40 $O/parity_$(basename $lib .so).log; exit 1; }
    echo "parity $lib: $(tail -1 $O/parity_$(basename $lib .so).log)"
done
bash tools/ab_wall.sh "C4 C5" $B $G > $O/wall_grid.txt 2>&1 || { tail $O/wall_grid.txt; exit 1; }
sed 's/strip=- bands=- //' $O/wall_grid.txt
bash tools/ab_wall.sh "C2 C3" $B $N $P $T > $O/wall_pk.txt 2>&1 || { tail $O/wall_pk.txt; exit 1; }
sed 's/strip=- bands=- //' $O/wall_pk.txt
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"
bash tools/pmc_ab.sh C4 "$PMC" $B $G > $O/pmc_C4.txt 2>&1 || { tail $O/pmc_C4.txt; exit 1; }
cat $O/pmc_C4.txt
bash tools/pmc_ab.sh C2 "$PMC" $B $P > $O/pmc_C2.txt 2>&1 || { tail $O/pmc_C2.txt; exit 1; }
cat $O/pmc_C2.txt
