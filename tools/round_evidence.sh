#!/bin/bash
# Round evidence on one GPU box, in one call: smoke, the GPU suite, the driver's bench command and
# the default bench line (both kept as gpurun_out/*.log), then PMC + kernel traces per config
# (tools/profile_round.sh).  Stops at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
    local name=$1 limit=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc: $(grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 1 | cut -c1-200)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
echo "nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 20
step bench_default 300 python bench.py --no-cpu-baseline --also C3,C4,C5
bash tools/profile_round.sh ${CONFIGS:-C2 C3 C4 C5}
