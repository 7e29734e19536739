#!/bin/bash
# Round-end evidence on the GPU box, per config: PMC passes (tools/pmc.sh) -> summary and
# gpurun_out/pmc_traffic.json; then the bench line of the config under
# rocprofv3 --kernel-trace --stats (the same process: its kernel_avg_ms and the trace's average
# duration of the trace kernel describe the same launches; no Tick probe, no work count, so
# every dispatch of that kernel is a bench launch: warm-up, the 16 timed launches, then the 16 of
# bench.py's untimed per-launch-event pass), reconciled by tools/trace_summary.py.
#   bash tools/profile_round.sh C2 C3 C4 C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json 2>/dev/null
for cfg in "$@"; do
    rm -rf "gpurun_out/pmc_$cfg"
    bash tools/pmc.sh "$cfg" > "gpurun_out/pmc_$cfg.log" 2>&1 || { echo "pmc $cfg failed"; exit 1; }
    python3 tools/pmc_summary.py "gpurun_out/pmc_$cfg" --json gpurun_out/pmc_traffic.json --config "$cfg" \
        --frames-per-launch 64 > "gpurun_out/pmc_${cfg}_summary.txt"
    rm -rf "gpurun_out/trace_$cfg"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/trace_$cfg" -o run \
        -- python3 bench.py --config "$cfg" --also "" --no-cpu-baseline --no-tick --pmc gpurun_out/pmc_traffic.json \
        > "gpurun_out/trace_bench_$cfg.json" 2> "gpurun_out/trace_$cfg.log"
    rc=$?; echo "trace $cfg rc=$rc: $(tail -c 200 gpurun_out/trace_bench_$cfg.json)"; [ $rc -eq 0 ] || exit $rc
    find "gpurun_out/trace_$cfg" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/trace_${cfg}_kernel_stats.csv" \;
    python3 tools/trace_summary.py "gpurun_out/trace_$cfg" --last 16 --skip-last 16 \
        --bench "gpurun_out/trace_bench_$cfg.json" > "gpurun_out/trace_${cfg}_reconcile.txt"
done
