#!/bin/bash
# Round-end check of the product build on one MI355X (GPU box, through gpurun):
#   bash tools/round_check.sh OUT_DIR [steps]
# the GPU suite, smoke, the driver's own bench command (--gpus 1 --steps 20 --warmup 5) and the default
# bench line (1024 frames, also C2/C4/C5, CPU baseline, Tick rates), each under its own time limit; prints
# one summary line per bench run.  (Round 4's one-off drivers tools/rounds/r04b.sh ... r04z.sh, which the
# r04 profiles cite, were this script with fixed output directories; git history keeps them.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=${1:-gpurun_out/check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=15 > $O/gpu.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $O/gpu.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu.log)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || { tail $O/driver.err; exit 1; }
timeout -k 10 500 python bench.py ${2:+--steps $2} > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
for f in driver bench; do
python3 - $O/$f.json $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["config"]["workload"].split(":")[0]
print(sys.argv[2], w, round(d["value"] / 1e3, 1), "Gray/s", round(d["ms_per_step"] * 1e3, 2), "us/frame; single",
      round(d.get("single_launch_fps", 0)), "tick", round(d.get("tick_fps_incl_d2h", 0)), "async",
      round(d.get("tick_async_fps_incl_d2h", 0)), "roofline", round(d["roofline"]["frac"], 4), "valu",
      round(d["roofline_valu"]["frac"] or 0, 3), "order", d.get("dispatch_order"))
for k, v in d.get("also", {}).items():
    lone = v.get("lone_frame") or {}
    print("  ", k, round(v["value"] / 1e3, 1), "Gray/s", round(v["ms_per_step"] * 1e3, 2), "us/frame",
          f"lone {lone['single_launch_ms'] * 1e3:.1f} us (order {lone['dispatch_order']})" if lone else "")
for k, v in (d.get("tick_by_config") or {}).items():
    if isinstance(v, dict):
        print("   tick", k, round(v["tick_fps"], 1), "fps sync", round(v["tick_async_fps"], 1), "async",
              round(v["tick_d2h_gbs"], 1), "GB/s")
c = d["cpu_baseline"]
print("   cpu", round(c["value"], 1), c["frame_ms_p10_p50_p90"], c["cpus_scheduled"], c["cgroup_throttled"])
PY
done
