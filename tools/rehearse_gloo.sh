#!/bin/bash
# Multi-process rehearsal of bench.py's N > 1 path on a one-GPU box: N ranks share the GPU and the
# collectives run over gloo (--rehearse-gloo; RCCL refuses two ranks on one GPU).  Every run
# verifies rank 0's decoded frames against a single-launch render (--verify, exit 3 on a mismatch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
port=29611
for spec in "2 auto C2 --batch 16" "3 auto C3 --batch 8" "4 on C2 --batch 16" "4 off C3 --batch 16 --band-format rgb24" "2 auto C2 --batch 16 --rank0-codec" "3 on C4 --batch 8 --no-fuse"; do
    set -- $spec
    n=$1; comp=$2; cfg=$3; shift 3
    port=$((port + 1))
    log=gpurun_out/rehearse_${n}_${comp}_${cfg}.log
    timeout -k 10 240 python bench.py --gpus $n --rehearse-gloo --master-port $port --config $cfg --size 960x540 \
        --steps 96 --warmup 32 --compositor $comp --verify --no-cpu-baseline "$@" > $log 2>&1
    rc=$?
    echo "== N=$n compositor=$comp $cfg $* rc=$rc: $(grep -h '^{' $log | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read() or "{}"); print(d.get("n_gpus"), d.get("verified_frames"), round(d.get("ms_per_step",0)*1e3,1), "us/frame", d.get("config",{}).get("parallelism","")[:90])' 2>/dev/null)"
    if [ $rc -ne 0 ]; then tail -5 $log; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc; fi
done
