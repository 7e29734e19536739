#!/bin/bash
# Timing-only ablations (output wrong by design, never kept): wall per frame of each variant vs the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/ab_wall.sh "${AB_CFGS:-C4 C5 C3}" lib/libraytracer_hip.so $AB_LIBS > gpurun_out/r03_ablate.txt 2>&1
