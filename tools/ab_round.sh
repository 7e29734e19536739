#!/bin/bash
# GPU box: parity suite of the in-tree build, then an A/B by wall time per frame:
#   AB_LIBS="lib/ab/libraytracer_hip_X.so" AB_CFGS="C2 C3" bash tools/ab_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 gpurun_out/ab_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for lib in $AB_LIBS; do  # parity of every variant before timing it
    RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$lib" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
        -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1; rc=$?
    echo "parity $lib rc=$rc: $(tail -1 gpurun_out/ab_parity.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_wall.sh "${AB_CFGS:-C2 C3}" lib/libraytracer_hip.so $AB_LIBS | sed 's/strip=- bands=- //'
[ -n "${AB_EMPTY:-}" ] && EXTRA="--strip spheres,planes,lights" bash tools/ab_wall.sh C2 lib/libraytracer_hip.so $AB_LIBS | sed 's/bands=- //'
exit 0
