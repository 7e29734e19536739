#!/bin/bash
# Packed f32 sphere pairs in the direct kernel (in-tree, RT_PACKED_PAIRS=1) against the scalar pair loops
# (scalar) and the packed build capped at 80 SGPRs (pk80): parity of every build, wall C2/C3, PMC per C2 dispatch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03pk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in lib/ab/libraytracer_hip_pk80.so; do
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$lib" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
echo "parity $lib: $(tail -1 $O/parity.log)"
done
bash tools/ab_wall.sh "C2 C3" lib/ab/libraytracer_hip_scalar.so lib/libraytracer_hip.so lib/ab/libraytracer_hip_pk80.so > $O/wall.txt 2>&1 || exit 1
cat $O/wall.txt
bash tools/pmc_ab.sh C2 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
    lib/ab/libraytracer_hip_scalar.so lib/libraytracer_hip.so lib/ab/libraytracer_hip_pk80.so
