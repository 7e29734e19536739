#!/bin/bash
# GPU box, end of a change: smoke, the whole GPU suite, the bench line of every config, the
# one-process rehearsal of the N>1 path.  Each step under its own limit; stops at a crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
    local name=$1 limit=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc: $(grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 1 | cut -c1-220)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step bench_C2 300 python bench.py
for c in C3 C4 C5; do step bench_$c 300 python bench.py --config $c --no-cpu-baseline; done
DIST_RUNS="tiles:64 rgb24:8" step dist 300 bash tools/dist_rehearsal.sh
cat gpurun_out/dist.log
