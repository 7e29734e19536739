#!/bin/bash
# r04: the product build end to end -- the GPU suite, smoke, the default bench line -- then single-frame
# launches with 8 tiles per workgroup (w8) against the product's 4, and the bundle kernel's ablations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
tail -1 $O/gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2", round(d["value"] / 1e3, 1), "Gray/s", round(d["ms_per_step"] * 1e3, 2), "us/frame; single", round(d["single_launch_fps"]),
      "tick", round(d["tick_fps_incl_d2h"]), "async", round(d["tick_async_fps_incl_d2h"]))
for k, v in d.get("also", {}).items():
    print(k, round(v["value"] / 1e3, 1), "Gray/s", round(v["ms_per_step"] * 1e3, 2), "us/frame")
c = d["cpu_baseline"]
print("cpu", round(c["value"], 1), c["frame_ms_p10_p50_p90"], c["cpus_scheduled"], c["cgroup_throttled"])
PY
for rep in 1 2; do for c in C2 C3; do for lib in lib/libraytracer_hip.so lib/ab/libraytracer_hip_w8.so; do
    timeout -k 10 120 python tools/frame_wall.py --config $c --batch 1 --frames 400 --lib uu-infogr-raytracer_amd/$lib \
        2>&1 | grep -v amdgpu.ids | sed 's/strip=- bands=- //' || exit 1
done; done; done
bash tools/rounds/r04_ablate.sh || exit 1
