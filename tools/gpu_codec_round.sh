#!/bin/bash
# GPU box: codec parity tests, then the N>1 data path rehearsed in one process (--dist-path)
# for each band format, then a kernel-trace profile of the tile-encoded path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/codec_gpu.log 2>&1; rc=$?
echo "codec rc=$rc"; tail -3 gpurun_out/codec_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${DIST_RUNS:-tiles:8 tiles:16 rgb24:8}; do
  fmt=${cfg%%:*}; b=${cfg##*:}
  timeout -k 10 200 python bench.py --dist-path --band-format $fmt --batch $b --steps 400 --warmup 100 --no-cpu-baseline > gpurun_out/dist_${fmt}_$b.json 2> gpurun_out/dist_${fmt}_$b.err; rc=$?
  echo "dist $fmt batch $b rc=$rc"; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2),'us/frame', d['config'].get('gather_wire_bytes_per_frame'))" gpurun_out/dist_${fmt}_$b.json
  [ $rc -eq 0 ] || { tail -20 gpurun_out/dist_${fmt}_$b.err; exit $rc; }
done
if [ "${PROFILE:-1}" = "1" ]; then
  rm -rf gpurun_out/prof_tiles
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tiles -o run -- python3 bench.py --dist-path --band-format tiles --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_tiles.log 2>&1; rc=$?
  echo "prof rc=$rc"; find gpurun_out/prof_tiles -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \;
fi
