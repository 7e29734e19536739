#!/bin/bash
# r05ae: shadow grids in the direct kernel's shadow scans -- H (previous commit) against the working tree with the
# grids (default) and without (RT_SHADOW_GRID=0), C3 / C2, 64-frame launches; then the parity tests of the grids.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05ae
mkdir -p $O
for c in C3 C2; do
  for rep in 1 2; do
    for v in "H|1" "T|1" "T|0"; do
      lib=lib/libraytracer_hip.so; [ ${v%%|*} = H ] && lib=lib/ab/libraytracer_hip_H.so
      RT_SHADOW_GRID=${v#*|} timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 1024 --lib uu-infogr-raytracer_amd/$lib 2>&1 \
          | grep -v amdgpu.ids | sed "s/^/$v: /" >> $O/wall.txt || exit 1
    done
  done
done
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "golden or random or grid or stats" > $O/tests.log 2>&1 \
    || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
