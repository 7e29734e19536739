#!/bin/bash
# r05t: rt_set_counting (ABI 10) -- one-frame launches with the counters on / off (product) beside NC (the
# counters compiled out), then the GPU suite and the bench's default line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05t
mkdir -p $O
for c in C2 C3 C4; do
  for rep in 1 2; do
    for v in "lib/ab/libraytracer_hip_NC.so|" "lib/libraytracer_hip.so|" "lib/libraytracer_hip.so|--no-count"; do
      lib=${v%%|*}; ex=${v#*|}
      timeout -k 10 180 python tools/frame_wall.py --config $c --batch 1 --frames 1024 --lib uu-infogr-raytracer_amd/$lib $ex 2>&1 \
          | grep -v amdgpu.ids >> $O/wall_b1.txt || exit 1
    done
  done
done
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall_b1.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"][:40], round(d["value"] / 1e3, 1), "Gray/s", round(d["ms_per_step"] * 1e3, 2), "us/frame; single",
      round(d.get("single_launch_fps", 0)), "tick", round(d.get("tick_fps_incl_d2h", 0)), "async", round(d.get("tick_async_fps_incl_d2h", 0)))
for k, v in d.get("also", {}).items():
    print("  ", k, round(v["value"] / 1e3, 1), "Gray/s", round(v["ms_per_step"] * 1e3, 2), "us/frame")
for k, v in (d.get("tick_by_config") or {}).items():
    if isinstance(v, dict):
        print("   tick", k, round(v["tick_fps"], 1), "sync", round(v["tick_async_fps"], 1), "async", round(v["tick_d2h_gbs"], 1), "GB/s")
PY
