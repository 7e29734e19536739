#!/bin/bash
# r05w: which part of the measured-order change slows the lone-frame kernel: H (previous commit), T (working
# tree), Tv1 (wave index not readfirstlane'd), Tv2 (no tile-cost recording code), Tv3 (no tile_order read).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05w
mkdir -p $O
for c in "C2|1" "C3|2"; do
  export RT_DISPATCH_ORDER=${c#*|}
  for rep in 1 2; do
    for lib in lib/ab/libraytracer_hip_H.so lib/libraytracer_hip.so lib/ab/libraytracer_hip_Tv1.so lib/ab/libraytracer_hip_Tv2.so lib/ab/libraytracer_hip_Tv3.so; do
      timeout -k 10 120 python tools/frame_wall.py --config ${c%%|*} --batch 1 --frames 1024 --no-count --lib uu-infogr-raytracer_amd/$lib 2>&1 \
          | grep -v amdgpu.ids >> $O/wall.txt || exit 1
    done
  done
done
unset RT_DISPATCH_ORDER
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
