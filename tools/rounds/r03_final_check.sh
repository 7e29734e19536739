#!/bin/bash
# End-of-session check on one GPU box: smoke, the GPU suite, the driver's bench command, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03f
step() {
    local name=$1 limit=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/r03f/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc: $(grep -v amdgpu.ids "gpurun_out/r03f/$name.log" | tail -n 1 | cut -c1-200)"
    [ $rc -eq 0 ] || exit $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 400 python bench.py --no-cpu-baseline --also C3,C4,C5
