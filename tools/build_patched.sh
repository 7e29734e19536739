#!/bin/bash
# A/B build of the product kernels with a patch applied (CPU side, before gpurun):
#   tools/build_patched.sh NAME PATCH [extra hipcc flags]  ->  uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_NAME.so
set -e
NAME=$1; PATCH=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/uu-infogr-raytracer_amd/csrc
T=$(mktemp -d)
cp $C/rt_kernel.hip $C/*.h $T/
(cd $T && patch -s -p1 < $R/$PATCH)
make -s -C $C obj/rt_api.o obj/rt_codec.o >/dev/null 2>&1 || make -C $C $C/obj/rt_api.o $C/obj/rt_codec.o
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize"
/opt/rocm/bin/hipcc $F "$@" -I$R/include -c -o $T/k.o $T/rt_kernel.hip
mkdir -p $R/uu-infogr-raytracer_amd/lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o $R/uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_$NAME.so \
    $T/k.o $C/obj/rt_codec.o $C/obj/rt_api.o -ldl
rm -rf $T
echo built lib/ab/libraytracer_hip_$NAME.so
