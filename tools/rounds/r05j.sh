#!/bin/bash
# r05j: the forward walk of the bundle kernel split (timing-only ablations, tools/ablate/r05_fwd*.patch):
# fwd0 = forward walk only; f1 = its primary segment only; f2 = no exact tests on reflected segments;
# f3 = no plane tests on reflected segments.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05j
mkdir -p $O
bash tools/ab_wall.sh "C4 C5" lib/ab/libraytracer_hip_fwd0.so lib/ab/libraytracer_hip_fwd_f1.so lib/ab/libraytracer_hip_fwd_f2.so lib/ab/libraytracer_hip_fwd_f3.so > $O/wall.txt 2>&1 || { tail $O/wall.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" lib/ab/libraytracer_hip_fwd0.so lib/ab/libraytracer_hip_fwd_f1.so lib/ab/libraytracer_hip_fwd_f2.so lib/ab/libraytracer_hip_fwd_f3.so > $O/pmc.txt 2>&1 || { tail $O/pmc.txt; exit 1; }
cat $O/pmc.txt
