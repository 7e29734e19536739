#!/bin/bash
# A/B build of the product library with a patch applied (CPU side, before gpurun):
#   tools/build_patched.sh NAME PATCH [extra hipcc flags]  ->  $ABDIR/libraytracer_hip_NAME.so
# ABDIR defaults to uu-infogr-raytracer_amd/lib/ab, which .gpurunignore keeps off the GPU box; builds a GPU run
# needs go to ABDIR=uu-infogr-raytracer_amd/lib/probe (shipped; emptied after the run).
# The patch (-p1, paths relative to csrc/) may touch rt_kernel.hip, rt_api.cpp and the headers; the
# objects of untouched sources come from the product build.
set -e
NAME=$1; PATCH=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/uu-infogr-raytracer_amd/csrc
T=$(mktemp -d)
mkdir -p $T/x/csrc
ln -s $R/include $T/include   # rt_api.cpp includes ../../include/raytracer_hip.h
cp $C/rt_kernel.hip $C/rt_api.cpp $C/*.h $T/x/csrc/
(cd $T/x/csrc && patch -s -p1 < $R/$PATCH)
make -s -C $C obj/rt_api.o obj/rt_codec.o >/dev/null 2>&1 || make -C $C $C/obj/rt_api.o $C/obj/rt_codec.o
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero"
/opt/rocm/bin/hipcc $F -fno-slp-vectorize "$@" -I$R/include -c -o $T/k.o $T/x/csrc/rt_kernel.hip
API=$C/obj/rt_api.o
changed=0
for f in rt_api.cpp $(cd $C && ls *.h); do cmp -s $C/$f $T/x/csrc/$f || changed=1; done
if [ $changed = 1 ]; then  # rt_api.cpp or a header it includes (record layouts) changed
    /opt/rocm/bin/hipcc $F "$@" -x hip -c -o $T/api.o $T/x/csrc/rt_api.cpp
    API=$T/api.o
fi
D=$R/${ABDIR:-uu-infogr-raytracer_amd/lib/ab}
mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o $D/libraytracer_hip_$NAME.so \
    $T/k.o $C/obj/rt_codec.o $API -ldl
rm -rf $T
echo built $D/libraytracer_hip_$NAME.so
