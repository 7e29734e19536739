#!/bin/bash
# GPU-box run: smoke -> pytest -m gpu -> bench, each under its own time limit.
# Stops at the first step that crashed, timed out or shows a GPU fault (test failures
# alone do not stop the chain).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
    local name=$1 limit=$2; shift 2
    echo "== $name (limit ${limit}s)"
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || grep -qiE "memory access fault|hsa_status|segmentation|core dumped|hipErrorLaunchFailure|illegal" "gpurun_out/$name.log"; }; then
        echo "== stopping after $name"
        exit $rc
    fi
    return 0
}
step smoke 420 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
step bench 600 python bench.py "$@"
if [ "${PROFILE:-0}" = "1" ]; then
    export TMPDIR=/tmp
    step profile 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
        -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline "$@"
    find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \;
fi
for cfg in ${BENCH_CONFIGS:-}; do
    step "bench_$cfg" 600 python bench.py --config "$cfg" --no-cpu-baseline --steps 50
done
