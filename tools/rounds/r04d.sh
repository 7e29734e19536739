#!/bin/bash
# r04: single-frame launches with 2 / 4 tiles per workgroup (lib/ab/libraytracer_hip_w2 / _w4; mg1 = one wave per
# workgroup, the same code otherwise): parity, then wall per frame of back-to-back rt_render_device launches (C2,
# C3, the empty C2 scene) and the batched shape beside them (unchanged launch), alternating builds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04d
mkdir -p $O
M1=lib/ab/libraytracer_hip_mg1.so
W2=lib/ab/libraytracer_hip_w2.so
W4=lib/ab/libraytracer_hip_w4.so
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$W4" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity_w4.log 2>&1 || { echo "PARITY FAILED $W4"; tail -40 $O/parity_w4.log; exit 1; }
echo "parity $W4: $(tail -1 $O/parity_w4.log)"
for rep in 1 2; do
    for c in "C2" "C3" "C2 --strip spheres,planes,lights"; do
        for lib in $M1 $W2 $W4; do
            timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 --lib uu-infogr-raytracer_amd/$lib \
                2>&1 | grep -v amdgpu.ids | sed 's/bands=- //' || exit 1
        done
    done
done
W4B=lib/ab/libraytracer_hip_w4b.so  # 4 tiles per workgroup for batch launches too
RAYTRACER_HIP_LIB="$PWD/uu-infogr-raytracer_amd/$W4B" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity_w4b.log 2>&1 || { echo "PARITY FAILED $W4B"; tail -40 $O/parity_w4b.log; exit 1; }
for rep in 1 2; do for c in C2 C3; do for lib in $M1 $W4B; do
    timeout -k 10 120 python tools/frame_wall.py --config $c --batch 64 --frames 1024 --lib uu-infogr-raytracer_amd/$lib \
        2>&1 | grep -v amdgpu.ids | sed "s/strip=- bands=- //" || exit 1
done; done; done
# the N > 1 pipeline rehearsed with one rank: the default path (rank 0 renders into its frames: a world of one
# exchanges nothing now) and the shipping rank's shape (--rank0-codec), each verified, then stage tables
for f in "" "--rank0-codec"; do
    timeout -k 10 180 python bench.py --dist-path $f --steps 20 --warmup 5 --also-dist "" --no-cpu-baseline > $O/dist$f.json \
        2> $O/dist$f.err || { tail $O/dist$f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step']*1e3,2), 'us/frame, verified', d.get('verified_frames'))" $O/dist$f.json "dist-path $f"
done
DIST_FLAGS="--no-verify" DIST_OUT=r04_dist_direct bash tools/dist_trace.sh || exit 1
DIST_FLAGS="--rank0-codec --no-verify" DIST_OUT=r04_dist_codec bash tools/dist_trace.sh || exit 1
head -12 gpurun_out/r04_dist_direct/stages.txt
head -30 gpurun_out/r04_dist_codec/stages.txt
