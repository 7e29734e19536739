#!/bin/bash
# GPU box: per-batch overhead of the N>1 tile pipeline, rehearsed in one process (bench.py
# --dist-path --rank0-codec: trace, encode, size all_reduce, gather, decode), at frame sizes
# where the trace is negligible (64x64) or a rank's share of 1080p at N = 8 (1920x136), for
# several frames per gather.  Prints us/frame and the host issue time per frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for size in ${SIZES:-64x64 1920x136}; do
  for b in ${BATCHES:-16 64}; do
    out=gpurun_out/ovh_${size}_$b.json
    timeout -k 10 120 python bench.py --dist-path --rank0-codec --band-format tiles --batch $b --size $size \
        --steps ${STEPS:-2048} --warmup 256 --no-cpu-baseline --no-tick > $out 2> ${out%.json}.err || { tail -5 ${out%.json}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'batch', sys.argv[3], 'period', round(d['ms_per_step']*1e3,2),'us/frame host', round(d['host_ms_per_step']*1e3,2), 'us/frame')" $out $size $b
  done
  timeout -k 10 120 python bench.py --size $size --steps ${STEPS:-2048} --warmup 256 --no-cpu-baseline --no-tick > gpurun_out/ovh_${size}_n1.json 2>/dev/null &&
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=1 path period', round(d['ms_per_step']*1e3,2),'us/frame')" gpurun_out/ovh_${size}_n1.json $size
done
