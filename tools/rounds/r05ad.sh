#!/bin/bash
# r05ad: where a direct-kernel frame goes (C2, C3): the product against timing-only ablations
# (tools/ablate/r05_d_*.patch), 64-frame launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05ad
mkdir -p $O
bash tools/ab_wall.sh "C3 C2" lib/libraytracer_hip.so lib/ab/libraytracer_hip_d_noshadow.so lib/ab/libraytracer_hip_d_walkonly.so \
    lib/ab/libraytracer_hip_d_fwd.so lib/ab/libraytracer_hip_d_fwd_f1.so > $O/wall.txt 2>&1 || { tail $O/wall.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
