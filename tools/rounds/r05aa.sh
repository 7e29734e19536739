#!/bin/bash
# r05aa: the bundle kernel's measured tile order -- its GPU tests; one-frame launches under the library's own
# choice (counters off) against H; batch launches with RT_BUNDLE_TILE_ORDER=2 (A/B) against the natural order.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "dispatch_order or tile_order or lone_frame_orders or counting" > $O/tests.log 2>&1 \
    || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for c in C4 C5; do
  n=$([ $c = C5 ] && echo 256 || echo 1024)
  for rep in 1 2; do
    timeout -k 10 180 python tools/frame_wall.py --config $c --batch 1 --frames $n --no-count --lib uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_H.so 2>&1 | grep -v amdgpu.ids | sed "s/^/lone H: /" >> $O/wall.txt || exit 1
    timeout -k 10 180 python tools/frame_wall.py --config $c --batch 1 --frames $n --no-count 2>&1 | grep -v amdgpu.ids | sed "s/^/lone auto: /" >> $O/wall.txt || exit 1
    for v in 0 2; do
      RT_BUNDLE_TILE_ORDER=$v timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 1024 2>&1 | grep -v amdgpu.ids | sed "s/^/batch order=$v: /" >> $O/wall.txt || exit 1
    done
  done
done
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
