#!/bin/bash
# GPU box: per-rank trace cost of an N-rank world (tools/frame_wall.py --bands R/N, two launches
# in flight; --batch F frames per launch) -- the compute side of the N > 1 scaling.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in "" 0/2 0/8; do
  for f in 1 16; do
    timeout -k 10 120 python tools/frame_wall.py --config ${CFG:-C2} --inflight 2 --frames 640 --batch $f ${b:+--bands $b} 2>&1 | grep -v amdgpu.ids
  done
done
