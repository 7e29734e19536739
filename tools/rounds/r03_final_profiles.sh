#!/bin/bash
# Final-build evidence: PMC summaries + kernel traces reconciled with the bench lines (C2-C5), then the one-process
# rehearsal of the N>1 path at the driver's shape (world 1 over RCCL: the library communicator path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03p
bash tools/profile_round.sh C2 C3 C4 C5 || exit $?
timeout -k 10 300 python bench.py --dist-path --steps 20 --warmup 5 --verify > gpurun_out/r03p/distpath.json 2> gpurun_out/r03p/distpath.err || { tail -20 gpurun_out/r03p/distpath.err; exit 1; }
tail -c 600 gpurun_out/r03p/distpath.json
