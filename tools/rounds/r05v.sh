#!/bin/bash
# r05v: same-box A/B of one-frame launches (counters off): H = the previous commit's library (orders 0-2)
# against the working tree (orders 0-3, the measured tile order), fixed orders and the library's own choice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/${OUT:-r05v}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "dispatch_order or tile_order or counting" > $O/tests.log 2>&1 \
    || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for c in C2 C3; do
  for rep in 1 2; do
    for v in "H|1" "H|2" "H|auto" "T|1" "T|2" "T|3" "T|auto"; do
      lib=lib/libraytracer_hip.so; [ ${v%%|*} = H ] && lib=lib/ab/libraytracer_hip_H.so
      o=${v#*|}
      if [ $o = auto ]; then unset RT_DISPATCH_ORDER; else export RT_DISPATCH_ORDER=$o; fi
      timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 1024 --no-count --lib uu-infogr-raytracer_amd/$lib 2>&1 \
          | grep -v amdgpu.ids | sed "s/^/${v%%|*} order $o: /" >> $O/wall.txt || exit 1
    done
  done
done
unset RT_DISPATCH_ORDER
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
