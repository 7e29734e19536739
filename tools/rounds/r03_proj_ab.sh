#!/bin/bash
# Lane-parallel light-frame projections in the merged shadow pass's cull (in-tree, RT_LANE_PROJ=1) against the
# uniform dots (base): parity of the in-tree build, wall C4/C5, PMC per C4 dispatch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03pj
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_wall.sh "C4 C5" lib/ab/libraytracer_hip_base.so lib/libraytracer_hip.so > $O/wall.txt 2>&1 || exit 1
cat $O/wall.txt
bash tools/pmc_ab.sh C4 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
    lib/ab/libraytracer_hip_base.so lib/libraytracer_hip.so
