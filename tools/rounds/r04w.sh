#!/bin/bash
# r04: PMC + kernel-trace reconciliation of C4 / C5 on the final build (the bundle kernel changed last).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/profile_round.sh C4 C5 || exit 1
for cfg in C4 C5; do cat gpurun_out/trace_${cfg}_reconcile.txt; done
