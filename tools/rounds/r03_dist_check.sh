#!/bin/bash
# The N > 1 pipeline rehearsed in one process (RCCL world of 1, rank 0 through the codec), the driver's 20-step shape:
# library collectives (default) vs torch.distributed, C2 and the C5 also-dist leg, every frame verified; then the
# stage trace of the default.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03d
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --dist-path --rank0-codec --steps 20 --warmup 5 --verify > $O/lib.json 2> $O/lib.err
timeout -k 10 300 python3 -u bench.py --dist-path --rank0-codec --steps 20 --warmup 5 --verify --torch-collectives > $O/torch.json 2> $O/torch.err
timeout -k 10 300 python3 -u bench.py --dist-path --steps 20 --warmup 5 --verify > $O/lib_direct.json 2> $O/lib_direct.err
bash tools/dist_trace.sh
cp gpurun_out/dist_trace/stages.txt $O/stages_lib.txt
