#!/bin/bash
# PMC passes over tools/codec_bench.py (world 1, C2), one counter group per run; summaries of
# the encode and decode kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_codec
rm -rf "$OUT"; mkdir -p "$OUT"
i=0
if [ -n "${PMC_GROUPS:-}" ]; then GROUPS_ARR=("$PMC_GROUPS"); else GROUPS_ARR=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
             "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"); fi
for group in "${GROUPS_ARR[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run \
        -- python3 tools/codec_bench.py --config C2 --worlds 1 --reps 3 > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$OUT/p$i.log"; }
    if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then exit $rc; fi
done
for k in encode_tiles decode_tiles encode_copy; do echo "== $k"; python3 tools/pmc_summary.py "$OUT" "$k"; done
