#!/bin/bash
# r04 second GPU call: shadow-grid A/B (parity + wall + PMC), the interactive-shape trace, and the
# N > 1 default path's stage table at HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/rounds/r04_grid_ab.sh || exit 1
mkdir -p gpurun_out/r04s && bash tools/rounds/r04_single_trace.sh > gpurun_out/r04s/summary.txt 2>&1 || { tail -20 gpurun_out/r04s/summary.txt; exit 1; }
cat gpurun_out/r04s/summary.txt
DIST_FLAGS="" DIST_OUT=r04_dist_direct bash tools/dist_trace.sh || exit 1
head -30 gpurun_out/r04_dist_direct/stages.txt
