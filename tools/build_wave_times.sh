#!/bin/bash
# Builds lib/ab/libraytracer_hip_wt.so: the product kernels plus tools/wave_times.patch (each direct-kernel wave
# records its start time, duration and HW_ID/XCC_ID; rt_debug_wave_times reads them back).  CPU side, before gpurun.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/uu-infogr-raytracer_amd/csrc
T=$(mktemp -d)
cp $C/rt_kernel.hip $C/*.h $T/
(cd $T && patch -s -p1 < $R/tools/wave_times.patch)
make -s -C $C obj/rt_api.o obj/rt_codec.o >/dev/null 2>&1 || make -C $C $C/obj/rt_api.o $C/obj/rt_codec.o
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize"
/opt/rocm/bin/hipcc $F -I$R/include -c -o $T/k.o $T/rt_kernel.hip
mkdir -p $R/uu-infogr-raytracer_amd/lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o $R/uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_wt.so \
    $T/k.o $C/obj/rt_codec.o $C/obj/rt_api.o -ldl
rm -rf $T
echo built lib/ab/libraytracer_hip_wt.so
