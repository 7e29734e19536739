#!/bin/bash
# r04: a batch launch's last frame with its tile rows in the cost estimate's order (profiles/ab/r04_last_frame_order.patch,
# lib/ab/libraytracer_hip_lfo.so: the cheapest rows end the launch) against the product build: parity, then the
# driver's bench shape (--steps 20 --warmup 5: one 20-frame launch) and 20-frame launches back to back, C2 / C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04q
mkdir -p $O
L=uu-infogr-raytracer_amd/lib
LFO=$PWD/$L/ab/libraytracer_hip_lfo.so
RAYTRACER_HIP_LIB=$LFO timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 $O/parity.log; exit 1; }
echo "parity lfo: $(tail -1 $O/parity.log)"
for rep in 1 2 3 4; do
    for c in C2 C3; do
        for lib in $PWD/$L/libraytracer_hip.so $LFO; do
            RAYTRACER_HIP_LIB=$lib timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 5 --also "" --no-cpu-baseline \
                --no-tick > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
            python3 -c "import json,sys; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$(basename $lib)', '$c', 'driver shape', round(d['ms_per_step']*1e3, 3), 'us/frame', round(d['value']/1e3, 1), 'Gray/s')"
        done
    done
done
for c in C2 C3; do
    for lib in $L/libraytracer_hip.so $L/ab/libraytracer_hip_lfo.so; do
        timeout -k 10 120 python tools/frame_wall.py --config $c --batch 20 --frames 1000 --reps 5 --lib $lib \
            2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //; s/; dispatch order -1//' || exit 1
    done
done
bash tools/rounds/r04r.sh > gpurun_out/r04r.log 2>&1 || { echo "r04r failed"; tail -20 gpurun_out/r04r.log; exit 1; }; cat gpurun_out/r04r.log
