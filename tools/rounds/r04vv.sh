#!/bin/bash
# r04 round-end check of the product build (after the no-cull early-out of the trace bundles): the GPU suite, smoke, the driver's own bench command
# (--gpus 1 --steps 20 --warmup 5) and the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r04vv
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || { tail $O/driver.err; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
for f in driver bench; do
python3 - $O/$f.json $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "C2", round(d["value"] / 1e3, 1), "Gray/s", round(d["ms_per_step"] * 1e3, 2), "us/frame; single",
      round(d["single_launch_fps"]), "(20:", round(d["single_launch_fps_20"]), ") tick", round(d["tick_fps_incl_d2h"]),
      "async", round(d["tick_async_fps_incl_d2h"]), "roofline", round(d["roofline"]["frac"], 4), "valu", round(d["roofline_valu"]["frac"], 3))
for k, v in d.get("also", {}).items():
    print("  ", k, round(v["value"] / 1e3, 1), "Gray/s", round(v["ms_per_step"] * 1e3, 2), "us/frame")
c = d["cpu_baseline"]
print("   cpu", round(c["value"], 1), c["frame_ms_p10_p50_p90"], c["cpus_scheduled"], c["cgroup_throttled"])
PY
done
