#!/bin/bash
# Kernel + HIP-runtime trace of the N > 1 pipeline rehearsed in one process (RCCL world of 1, rank 0 through the codec),
# the driver's 20-step shape on C2; tools/dist_stages.py turns it into the per-stage table.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/dist_trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/dist_trace/prof -o dist \
    -- python3 -u $R/bench.py --dist-path --rank0-codec --steps 20 --warmup 5 --also-dist "" > $R/gpurun_out/dist_trace/bench.txt 2>&1
cd $R && python3 tools/dist_stages.py gpurun_out/dist_trace/prof > gpurun_out/dist_trace/stages.txt 2>&1
