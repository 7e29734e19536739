#!/bin/bash
# PMC passes on the trace kernel, one counter group per rocprofv3 run (gfx950 rules:
# FETCH_SIZE and WRITE_SIZE in separate passes; never combined with tracing domains).
# Usage (GPU box): bash tools/pmc.sh CONFIG [extra bench args]
# Every dispatch of the trace kernel is one 64-frame launch (the bench's shape: --steps and
# --warmup multiples of 64, no clock ramp, no Tick probe / work count), so
# pmc_summary.py --frames-per-launch 64 gives per-launch and per-frame counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-C2}; shift || true
OUT=gpurun_out/pmc_$CFG
mkdir -p "$OUT"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD TCP_TOTAL_CACHE_ACCESSES_sum" ; do
    i=$((i+1))
    echo "== pass $i: $group"
    timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run \
        -- python3 bench.py --config "$CFG" --steps ${PMC_STEPS:-128} --warmup 64 --min-warmup-ms 0 --also "" \
           --no-cpu-baseline --no-tick "$@" > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ] && grep -qiE "memory access fault|illegal|segmentation|core dumped" "$OUT/p$i.log"; then exit $rc; fi
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
done
