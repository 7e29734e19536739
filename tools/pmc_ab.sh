#!/bin/bash
# One PMC pass per library build on one config (tools/frame_wall.py, 20 frames), then the
# per-dispatch averages of the trace kernel side by side.  Usage (GPU box):
#   bash tools/pmc_ab.sh C2 "SQ_INSTS_VALU SQ_INSTS_SALU ..." lib/ab/libA.so lib/libraytracer_hip.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=$1; counters=$2; shift 2
i=0
for lib in "$@"; do
    i=$((i+1))
    out=gpurun_out/pmcab_${cfg}_$i
    rm -rf "$out"
    timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d "$out" -o run \
        -- python3 tools/frame_wall.py --config "$cfg" --frames 20 --reps 1 --lib "uu-infogr-raytracer_amd/$lib" > "$out.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -5 "$out.log"; exit $rc; }
    echo "== $lib"
    python3 tools/pmc_summary.py "$out" | grep -v "HBM\|utilisation"
done
