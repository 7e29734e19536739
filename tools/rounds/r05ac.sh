#!/bin/bash
# r05ac: the counting-sort tile order -- its GPU tests and one-frame launches of C3 / C4 / C5 (counters off).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread --durations=8 -k "dispatch_order or tile_order or lone_frame_orders or counting" > $O/tests.log 2>&1 \
    || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
grep -A10 "slowest" $O/tests.log | head -12; echo "tests: $(tail -1 $O/tests.log)"
for c in C3 C4 C5; do
  n=$([ $c = C5 ] && echo 256 || echo 1024)
  timeout -k 10 180 python tools/frame_wall.py --config $c --batch 1 --frames $n --no-count 2>&1 | grep -v amdgpu.ids >> $O/wall.txt || exit 1
done
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
