#!/bin/bash
# r04 A/B: the level-0 ball cull with hoisted light-independent terms (the product build) against
# lib/ab/libraytracer_hip_nofm.so (the per-light cull of shadow_members): parity, wall C4/C5, PMC per C4 frame.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04g2
mkdir -p $O
F=lib/ab/libraytracer_hip_nofm.so  # the per-light cull of shadow_members at level 0 (the product: hoisted)
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$F" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity_nofm.log 2>&1 || { echo "PARITY FAILED $F"; tail -40 $O/parity_nofm.log; exit 1; }
echo "parity $F: $(tail -1 $O/parity_nofm.log)"
bash tools/ab_wall.sh "C4 C5" lib/libraytracer_hip.so $F 2>&1 | sed 's/strip=- bands=- //' || exit 1
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" \
    lib/libraytracer_hip.so $F || exit 1
