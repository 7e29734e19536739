#!/bin/bash
# Shadow-test lane slots of the bundle kernel by category and fold level (C4, C5), plus the kernel trace of the C4
# bench leg; tools/shadow_slots.py with the RT_SHADOW_CAT=1 build.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03s
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u tools/shadow_slots.py --configs C4 > $O/shadow_slots.txt 2>&1
