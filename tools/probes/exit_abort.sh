#!/bin/bash
# r06: the exit abort of r05b, one cause: every probe sequence (tools/probes/exit_abort_probe.py) in a process of
# its own, under the product build and the two pre-fix variants (built on the CPU side first:
#   ABDIR=uu-infogr-raytracer_amd/lib/probe tools/build_patched.sh rtld_global tools/probes/rtld_global.patch
#   ABDIR=uu-infogr-raytracer_amd/lib/probe tools/build_patched.sh pitched tools/probes/pitched_pageable.patch), exit status and stderr markers of each.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=${1:-gpurun_out/exit_abort}
mkdir -p $O
for lib in product rtld_global pitched; do
  L=uu-infogr-raytracer_amd/lib/libraytracer_hip.so
  [ $lib != product ] && L=uu-infogr-raytracer_amd/lib/probe/libraytracer_hip_$lib.so
  for s in ${SEQS:-A B C D E F G H I}; do
    RT_PROBE_PITCHED=1 RAYTRACER_HIP_LIB=$R/$L timeout -k 10 120 python tools/probes/exit_abort_probe.py $s > $O/${lib}_$s.log 2>&1
    rc=$?
    echo "$lib $s rc=$rc done=$(grep -c 'done' $O/${lib}_$s.log) double_free=$(grep -ci 'double free\|corrupt' $O/${lib}_$s.log)"
    [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
  done
done
exit 0
