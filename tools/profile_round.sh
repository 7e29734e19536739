#!/bin/bash
# Round-end evidence on the GPU box: PMC passes (tools/pmc.sh) and rocprofv3 kernel-trace
# summaries of bench.py for the given configs.  Usage: bash tools/profile_round.sh C2 C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "$@"; do
    steps=20; [ "$cfg" = "C4" ] || [ "$cfg" = "C5" ] && steps=5
    PMC_STEPS=$steps bash tools/pmc.sh "$cfg" || exit $?
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/trace_$cfg" -o run \
        -- python3 bench.py --config "$cfg" --steps 50 --warmup 5 --no-cpu-baseline > "gpurun_out/trace_$cfg.log" 2>&1
    rc=$?; echo "trace $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
