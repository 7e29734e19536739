#!/bin/bash
# A/B build of the whole library (kernels + host) from a copy of csrc/ with a sed expression applied to
# rt_internal.h (CPU side, before gpurun):
#   tools/build_full_variant.sh NAME 'sed expression'  ->  uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_NAME.so
set -e
NAME=$1; EXPR=$2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/uu-infogr-raytracer_amd/csrc
B=$(mktemp -d)
T=$B/pkg/csrc  # the sources include ../../include/raytracer_hip.h
mkdir -p $T && ln -s $R/include $B/include
cp $C/*.hip $C/*.cpp $C/*.h $T/
sed -i "$EXPR" $T/rt_internal.h
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -I$R/include"
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -c -o $T/k.o $T/rt_kernel.hip &
/opt/rocm/bin/hipcc $F -c -o $T/c.o $T/rt_codec.hip &
/opt/rocm/bin/hipcc $F -x hip -c -o $T/a.o $T/rt_api.cpp &
wait
mkdir -p $R/uu-infogr-raytracer_amd/lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o $R/uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_$NAME.so \
    $T/k.o $T/c.o $T/a.o -ldl
rm -rf $B
echo built lib/ab/libraytracer_hip_$NAME.so
