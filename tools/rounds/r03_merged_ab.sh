#!/bin/bash
# A/B of the merged shadow pass builds against the per-light passes (lib/ab/libraytracer_hip_base.so = HEAD before it):
# parity of each variant, wall per frame C4/C5, SALU/VALU/SMEM per dispatch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L="${AB_LIBS:-lib/ab/libraytracer_hip_base.so lib/ab/libraytracer_hip_merged2.so lib/ab/libraytracer_hip_merged4.so}"
AB_LIBS="$L" AB_CFGS="C4 C5" bash tools/ab_round.sh > gpurun_out/r03_merged_ab.txt 2>&1 || exit $?
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
    lib/libraytracer_hip.so $L >> gpurun_out/r03_merged_ab.txt 2>&1
