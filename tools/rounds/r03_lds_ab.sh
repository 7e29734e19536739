#!/bin/bash
# A/B: the bundle kernel's sphere table staged in LDS (RT_LDS_SCENE=1) vs scalar loads; parity of the variant,
# wall per frame on C4/C5, and SALU/SMEM/VALU/LDS instruction counts per dispatch (one PMC pass per build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB_LIBS="lib/ab/libraytracer_hip_ldsscene.so" AB_CFGS="C4 C5" bash tools/ab_round.sh > gpurun_out/r03_lds_ab.txt 2>&1 || exit $?
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
    lib/libraytracer_hip.so lib/ab/libraytracer_hip_ldsscene.so >> gpurun_out/r03_lds_ab.txt 2>&1
