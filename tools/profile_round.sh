#!/bin/bash
# Round-end evidence on the GPU box, per config: PMC passes (tools/pmc.sh) -> summary and
# gpurun_out/pmc_traffic.json; rocprofv3 --kernel-trace --stats of bench.py; then the bench
# line itself (reading that PMC summary for roofline.traffic / roofline_valu).
#   bash tools/profile_round.sh C2 C3 C4 C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json 2>/dev/null
for cfg in "$@"; do
    steps=32; [ "$cfg" = "C4" ] || [ "$cfg" = "C5" ] && steps=16
    rm -rf "gpurun_out/pmc_$cfg"
    PMC_STEPS=$steps bash tools/pmc.sh "$cfg" > "gpurun_out/pmc_$cfg.log" 2>&1 || { echo "pmc $cfg failed"; exit 1; }
    python3 tools/pmc_summary.py "gpurun_out/pmc_$cfg" --json gpurun_out/pmc_traffic.json --config "$cfg" \
        --frames-per-launch 16 > "gpurun_out/pmc_${cfg}_summary.txt"
    rm -rf "gpurun_out/trace_$cfg"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/trace_$cfg" -o run \
        -- python3 bench.py --config "$cfg" --steps 320 --warmup 64 --no-cpu-baseline --no-tick > "gpurun_out/trace_$cfg.log" 2>&1
    rc=$?; echo "trace $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
    extra=""; [ "$cfg" = "C2" ] || extra="--no-cpu-baseline"
    timeout -k 10 300 python3 bench.py --config "$cfg" --pmc gpurun_out/pmc_traffic.json $extra > "gpurun_out/bench_$cfg.json" 2> "gpurun_out/bench_$cfg.err"
    rc=$?; echo "bench $cfg rc=$rc: $(tail -c 300 gpurun_out/bench_$cfg.json)"; [ $rc -eq 0 ] || exit $rc
done
