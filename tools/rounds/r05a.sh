#!/bin/bash
# r05a: where the bundle kernel's C4/C5 frame goes at round start and the lone C4 frame
# (item 5).  Timing-only ablations built from tools/ablate/r05_*.patch (output wrong by design, never kept):
#   fwd = forward walk only (no fold), walkonly = the fold pops (re-walks) but shades nothing,
#   noshadow = no shadow pass, cull2 = the trace bundles' cull_mask computed twice (its cost = the increment).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05a
mkdir -p $O
L="lib/libraytracer_hip.so lib/ab/libraytracer_hip_abl_fwd.so lib/ab/libraytracer_hip_abl_walkonly.so lib/ab/libraytracer_hip_abl_noshadow.so lib/ab/libraytracer_hip_abl_cull2.so"
bash tools/ab_wall.sh "C4 C5" $L > $O/wall.txt 2>&1 || { tail $O/wall.txt; exit 1; }
cat $O/wall.txt
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" $L > $O/pmc.txt 2>&1 || { tail $O/pmc.txt; exit 1; }
cat $O/pmc.txt
for b in 1 8; do
  timeout -k 10 120 python tools/wave_times.py --lib uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_wt.so --config C4 --batch $b --reps 3 --map \
     --save $O/wt_C4_b$b.npz > $O/wt_C4_b$b.txt 2>&1 || { tail $O/wt_C4_b$b.txt; exit 1; }
  cat $O/wt_C4_b$b.txt
done
