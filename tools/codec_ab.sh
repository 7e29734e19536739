#!/bin/bash
# GPU box: codec parity (in-tree build), then isolated codec timings of the in-tree build and of
# the builds in $AB_LIBS (RAYTRACER_HIP_LIB), alternating, two passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py tests/test_codec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/codec_gpu.log 2>&1; rc=$?
echo "codec tests rc=$rc: $(tail -1 gpurun_out/codec_gpu.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in "" ${AB_LIBS:-}; do
    echo "== ${lib:-in-tree}"
    RAYTRACER_HIP_LIB="${lib:+$PWD/uu-infogr-raytracer_amd/$lib}" timeout -k 10 200 python tools/codec_bench.py \
        --config ${CODEC_CFG:-C2} --worlds 1 2 8 --frames 16 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
