#!/bin/bash
# r05i: merged shadow loop A/B on C4/C5 against the product (plane skip): Mv2 = no per-light 2a check
# (timing only), Mv3 = light constants in two 16-byte scalar loads, Mv4 = two candidate spheres per iteration.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05i
mkdir -p $O
bash tools/ab_wall.sh "C4 C5" lib/libraytracer_hip.so lib/ab/libraytracer_hip_Mv2.so lib/ab/libraytracer_hip_Mv3.so lib/ab/libraytracer_hip_Mv4.so > $O/wall.txt 2>&1 || { tail $O/wall.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" lib/libraytracer_hip.so lib/ab/libraytracer_hip_Mv2.so lib/ab/libraytracer_hip_Mv4.so > $O/pmc.txt 2>&1 || { tail $O/pmc.txt; exit 1; }
cat $O/pmc.txt
