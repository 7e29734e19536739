#!/bin/bash
# Kernel + HIP-runtime trace of the N > 1 pipeline rehearsed in one process (RCCL world of 1, rank 0 through the codec),
# the driver's 20-step shape on C2; tools/dist_stages.py turns it into the per-stage table.
# DIST_FLAGS overrides the path flags (default --rank0-codec; "" = the default path: rank 0 traces into its frames).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=${DIST_OUT:-dist_trace}
mkdir -p $R/gpurun_out/$O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/$O/prof -o dist \
    -- python3 -u $R/bench.py --dist-path ${DIST_FLAGS---rank0-codec} --steps 20 --warmup 5 --also-dist "" > $R/gpurun_out/$O/bench.txt 2>&1
cd $R && python3 tools/dist_stages.py gpurun_out/$O/prof > gpurun_out/$O/stages.txt 2>&1
