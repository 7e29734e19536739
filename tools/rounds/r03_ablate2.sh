#!/bin/bash
# Timing-only ablations of the bundle kernel (variants built from patched copies, output wrong by design):
# noshadow = no shadow pass (every ray unblocked), walkonly = the fold pops every record but shades nothing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03a2
L="lib/ab/libraytracer_hip_abl_noshadow.so lib/ab/libraytracer_hip_abl_walkonly.so"
bash tools/ab_wall.sh "C4 C5" lib/libraytracer_hip.so $L > gpurun_out/r03a2/wall.txt 2>&1 || exit 1
cat gpurun_out/r03a2/wall.txt
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
    lib/libraytracer_hip.so $L
