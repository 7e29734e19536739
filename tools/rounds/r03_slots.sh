#!/bin/bash
# Lane-slot utilisation of the exact sphere tests (tools/slot_probe.py) and the shadow-slot categories per fold level
# (tools/shadow_slots.py) with the in-tree kernels (merged shadow pass).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03slots
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u tools/slot_probe.py --configs C2 C3 C4 C5 > $O/slot_probe.txt 2>&1
timeout -k 10 600 python3 -u tools/shadow_slots.py --configs C4 > $O/shadow_slots.txt 2>&1
