#!/bin/bash
# Shadow-queue variants: split bounds per chunk (qsplit), 7 waves per SIMD (73 VGPRs, no spill: q7, qsplit7)
# against the merged per-level pass (noqueue); parity of each variant, wall C4/C5, slots of qsplit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03q2
mkdir -p $O
L="lib/ab/libraytracer_hip_qsplit.so lib/ab/libraytracer_hip_q7.so lib/ab/libraytracer_hip_qsplit7.so"
for lib in $L; do
    RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$lib" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
        -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity $lib FAILED"; tail -20 $O/parity.log; exit 1; }
    echo "parity $lib: $(tail -1 $O/parity.log)"
done
bash tools/ab_wall.sh "C4 C5" lib/ab/libraytracer_hip_noqueue.so lib/libraytracer_hip.so $L > $O/wall.txt 2>&1 || exit 1
cat $O/wall.txt
A=uu-infogr-raytracer_amd/lib/ab
timeout -k 10 600 python3 -u tools/slot_probe.py --configs C4 C5 --base-lib $A/libraytracer_hip_qsplit.so \
    --slots-lib $A/libraytracer_hip_qs_slots.so --slots2-lib $A/libraytracer_hip_qs_slots2.so > $O/slot_probe.txt 2>&1 || exit 1
cat $O/slot_probe.txt
