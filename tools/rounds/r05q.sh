#!/bin/bash
# r05q: (1) A/B of the merged shadow loop's all-lights-ok instantiation: product (MERGED == 2 where the lights allow)
# against M1 (tools/ablate/r05_merged1_only.patch: MERGED == 1 always) on C4/C5; (2) the lone C4 frame against a
# batch of 8 under PMC (why frame 0 of a launch runs ~15 % more shader cycles at the same clock); (3) the rank-0
# share rehearsals at N = 3 / 8 with the event-timed probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
bash tools/ab_wall.sh "C4 C5" lib/ab/libraytracer_hip_M1.so lib/libraytracer_hip.so > $O/wall.txt 2>&1 || { tail $O/wall.txt; exit 1; }
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
SETA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
SETB="TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
for b in 1 8; do
  for set in A B; do
    ctr=$SETA; [ $set = B ] && ctr=$SETB
    out=$O/pmc_b${b}_$set
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $out -o run \
        -- python3 tools/frame_wall.py --config C4 --frames 24 --reps 1 --batch $b > $out.log 2>&1 || { echo "pmc b$b $set failed"; tail -5 $out.log; exit 1; }
    echo "== batch $b set $set"
    python3 tools/pmc_summary.py $out | grep -v "HBM\|utilisation"
  done
done
bash tools/rounds/r05n.sh || exit 1
