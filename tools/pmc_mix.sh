#!/bin/bash
# Dynamic instruction mix of the trace kernel (PMC, one counter group per rocprofv3 run, gfx950
# limits: at most 8 SQ_ counters per pass).  Usage (GPU box): bash tools/pmc_mix.sh CONFIG
# Then: python3 tools/pmc_summary.py gpurun_out/pmcmix_CONFIG  (per 64-frame dispatch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-C2}; shift || true
OUT=gpurun_out/pmcmix_$CFG
mkdir -p "$OUT"
i=0
for group in "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
             "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_SALU" \
             "SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES SQ_WAVES" ; do
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
