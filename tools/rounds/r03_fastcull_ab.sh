#!/bin/bash
# Shadow-cull members with the light-independent terms hoisted (in-tree, RT_FAST_MEMBERS=1) against the
# per-light shadow_sphere_cull (oldcull), and the shadow queue on top of it (qfast): parity, wall C4/C5, PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03fc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_qfast.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_q.log 2>&1 || { tail -30 $O/parity_q.log; exit 1; }
tail -1 $O/parity_q.log
bash tools/ab_wall.sh "C4 C5" lib/ab/libraytracer_hip_oldcull.so lib/libraytracer_hip.so lib/ab/libraytracer_hip_qfast.so > $O/wall.txt 2>&1 || exit 1
cat $O/wall.txt
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_FLAT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
    lib/ab/libraytracer_hip_oldcull.so lib/libraytracer_hip.so
