#!/bin/bash
# r04: measured single-frame dispatch order (rt_dispatch_order): the whole GPU suite, then wall per frame of
# back-to-back rt_render_device launches with the order measured (default) and with each candidate fixed
# (RT_DISPATCH_ORDER), C1 / C2 / C3 / REF 1280x720, then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu_tests.log)"
for rep in 1 2; do
    for c in C1 C2 C3 "REF --size 1280x720"; do
        for ro in auto 0 1 2; do
            echo -n "[order $ro] "
            if [ $ro = auto ]; then
                timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 --reps 3 2>&1 | grep -v amdgpu.ids \
                    | sed 's/strip=- bands=- //' || exit 1
            else
                RT_DISPATCH_ORDER=$ro timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 --reps 3 \
                    2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
            fi
        done
    done
done
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('C2', round(d['value']/1e3,1), 'Gray/s', round(d['ms_per_step']*1e3,2), 'us/frame; single', round(d['single_launch_fps']), '(20-frame runs', round(d['single_launch_fps_20']), ') tick', round(d['tick_fps_incl_d2h']), 'async', round(d['tick_async_fps_incl_d2h']))
for k, v in d.get('also', {}).items(): print(k, round(v['value']/1e3,1), 'Gray/s', round(v['ms_per_step']*1e3,2), 'us/frame')
"
