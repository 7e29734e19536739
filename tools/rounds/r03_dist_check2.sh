#!/bin/bash
# The N > 1 rehearsal (world 1) with the per-leg batch choice: C2 one batch (library collectives), C5 pipelined
# (batches of >= 1 ms of trace), every frame verified; rank 0 direct and through the codec.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03d2
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --dist-path --steps 20 --warmup 5 --verify > $O/direct.json 2> $O/direct.err
timeout -k 10 300 python3 -u bench.py --dist-path --rank0-codec --steps 20 --warmup 5 --verify > $O/codec.json 2> $O/codec.err
