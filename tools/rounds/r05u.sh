#!/bin/bash
# r05u: the measured tile order (dispatch-order candidate 3) -- its GPU tests, then one-frame launches
# (counters off) under each fixed order and the library's own choice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "dispatch_order or tile_order or counting" > $O/tests.log 2>&1 \
    || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for c in C2 C3 C1 REF; do
  for rep in 1 2; do
    for o in 0 1 2 3 auto; do
      if [ $o = auto ]; then unset RT_DISPATCH_ORDER; else export RT_DISPATCH_ORDER=$o; fi
      timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 1024 --no-count 2>&1 | grep -v amdgpu.ids \
          | sed "s/^/order $o: /" >> $O/wall.txt || exit 1
    done
  done
done
unset RT_DISPATCH_ORDER
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
