#!/bin/bash
# r05o: the merged shadow loop's all-lights-ok instantiation (MERGED == 2) against the previous product (P),
# then the lone C4 frame's wave times with the shader clock per wave, the rank-0 share rehearsals (tools/rounds/r05n.sh) and the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05o
mkdir -p $O
bash tools/ab_wall.sh "C4 C5" lib/ab/libraytracer_hip_P.so lib/libraytracer_hip.so > $O/wall.txt 2>&1 || { tail $O/wall.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
for b in 1 8; do
  timeout -k 10 120 python tools/wave_times.py --lib uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_wt.so --config C4 --batch $b --reps 3 \
      > $O/wt_C4_b$b.txt 2>&1 || { tail $O/wt_C4_b$b.txt; exit 1; }
  grep "frame\|clock\|medians" $O/wt_C4_b$b.txt
done
bash tools/rounds/r05n.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
