#!/bin/bash
# r05final: end-of-round check of the final build (tools/round_check.sh) and the N > 1 rehearsals (r05n).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/round_check.sh gpurun_out/r05final || exit 1
grep -A16 "slowest" gpurun_out/r05final/gpu.log | head -18
bash tools/rounds/r05n.sh || exit 1
