#!/bin/bash
# The driver's scaling commands (bench.py --gpus N --steps 20 --warmup 5, full 1920x1080 C2, defaults:
# compositor auto = on at N >= 8) rehearsed on a one-GPU box: N ranks share the GPU over gloo
# (--rehearse-gloo), rank 0's decoded frames checked against a single-launch render (--verify).
# Timings are N processes time-sharing one GPU: not results.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
port=29711
for n in ${RANKS:-2 4 8}; do
    port=$((port + 1))
    log=gpurun_out/rehearse_driver_$n.log
    timeout -k 10 300 python bench.py --gpus $n --rehearse-gloo --master-port $port --steps 20 --warmup 5 \
        --verify --no-cpu-baseline > $log 2>&1
    rc=$?
    echo "== N=$n rc=$rc: $(grep -h '^{' $log | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read() or "{}"); print(d.get("n_gpus"), "verified", d.get("verified_frames"), d.get("config",{}).get("parallelism","")[:140])' 2>/dev/null)"
    if [ $rc -ne 0 ]; then grep -v amdgpu.ids $log | tail -5; exit $rc; fi
done
