#!/bin/bash
# GPU box: the N>1 data path rehearsed in one process (bench.py --dist-path: RCCL world of 1,
# batched gathers, reassembly) per band format (tiles0 = tiles with --rank0-codec: rank 0's
# own bands through encode + decode too); prints us/frame and wire bytes per frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${DIST_RUNS:-tiles:8 tiles:16 rgb24:8}; do
  fmt=${cfg%%:*}; b=${cfg##*:}
  extra=""; [ "$fmt" = "tiles0" ] && { fmt=tiles; extra=--rank0-codec; }
  timeout -k 10 200 python bench.py --dist-path --band-format $fmt --batch $b $extra --steps ${STEPS:-600} --warmup 100 --no-cpu-baseline > gpurun_out/dist_${fmt}_$b.json 2> gpurun_out/dist_${fmt}_$b.err; rc=$?
  [ $rc -eq 0 ] || { echo "dist $fmt batch $b rc=$rc"; tail -20 gpurun_out/dist_${fmt}_$b.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'batch', sys.argv[3], round(d['ms_per_step']*1e3,2),'us/frame', d['config'].get('gather_wire_bytes_per_frame'))" gpurun_out/dist_${fmt}_$b.json $fmt $b
done
