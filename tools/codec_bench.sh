#!/bin/bash
# GPU box: codec parity tests, isolated codec timings (tools/codec_bench.py), and optionally
# their kernel-trace summary (PROFILE=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/codec_gpu.log 2>&1; rc=$?
echo "codec tests rc=$rc"; tail -3 gpurun_out/codec_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/codec_bench.py --config ${CODEC_CFG:-C2} --worlds 1 2 8 > gpurun_out/codec_bench.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/codec_bench.txt; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-0}" = "1" ]; then
  rm -rf gpurun_out/prof_codec
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_codec -o run -- python3 tools/codec_bench.py --config C2 --worlds 1 > gpurun_out/prof_codec.log 2>&1; rc=$?
  find gpurun_out/prof_codec -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | grep -v Fill
fi
exit $rc
