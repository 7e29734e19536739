#!/bin/bash
# r04 round-end evidence: PMC + kernel-trace reconciliation per config at the bench's long shape
# (tools/profile_round.sh), then the driver's shape (--steps 20 --warmup 5: one 20-frame launch per
# config, the timed one, then the untimed per-launch-event pass) for C2 and C4 under rocprofv3 --stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/profile_round.sh C2 C3 C4 C5 || exit 1
export TMPDIR=/tmp
for cfg in C2 C4; do
    rm -rf gpurun_out/dtrace_$cfg
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dtrace_$cfg -o run \
        -- python3 bench.py --config $cfg --steps 20 --warmup 5 --also "" --no-cpu-baseline --no-tick \
        > gpurun_out/dtrace_bench_$cfg.json 2> gpurun_out/dtrace_$cfg.log || { tail gpurun_out/dtrace_$cfg.log; exit 1; }
    find gpurun_out/dtrace_$cfg -name "*kernel_stats.csv" -exec cp {} gpurun_out/dtrace_${cfg}_kernel_stats.csv \;
    python3 tools/trace_summary.py gpurun_out/dtrace_$cfg --last 1 --skip-last 1 --bench gpurun_out/dtrace_bench_$cfg.json \
        > gpurun_out/dtrace_${cfg}_reconcile.txt || exit 1
    cat gpurun_out/dtrace_${cfg}_reconcile.txt
done
for cfg in C2 C3 C4 C5; do cat gpurun_out/trace_${cfg}_reconcile.txt; done
bash tools/rounds/r04h.sh > gpurun_out/r04h.log 2>&1 || { tail -20 gpurun_out/r04h.log; exit 1; }
bash tools/rounds/r04i.sh > gpurun_out/r04i.log 2>&1 || { tail -20 gpurun_out/r04i.log; exit 1; }
