#!/bin/bash
# r04: the interactive shape (one frame per launch, rt_render_device, C2) -- wall per frame, then a
# kernel trace split into dispatch duration and inter-dispatch gap; the empty scene (launch cost
# alone) and device-memory kernargs beside it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04s
mkdir -p $O
cd $R
for e in "" "HIP_FORCE_DEV_KERNARG=1"; do
  for s in "" "spheres,planes,lights"; do
    echo -n "[$e] "
    env $e timeout -k 10 120 python tools/frame_wall.py --config C2 --batch 1 --frames 400 ${s:+--strip $s} 2>&1 \
      | grep -v amdgpu.ids || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for s in "" "spheres,planes,lights"; do
  d=$O/kt${s:+_empty}
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
    -- python3 $R/tools/frame_wall.py --config C2 --batch 1 --frames 200 --reps 1 ${s:+--strip $s} > $d.log 2>&1 || { tail $d.log; exit 1; }
  (cd $R && python3 tools/single_gap.py $d --last 200) || exit 1
done
