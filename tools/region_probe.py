"""Where the fixed cost of a short timed region goes (bench.py's N = 1 region at the driver's
--steps 20: one launch of 20 frames between two torch.cuda.synchronize() calls).
Per repetition: sync | t0 | ev0.record | t1 | render_bands_batch(F frames) | t2 | ev1.record |
t3 | sync | t4; medians of each host segment, of the wall, of ev0->ev1 and of the launch's own
event pair (rt_set_timing 1), with and without the per-launch timing events.
    python tools/region_probe.py [--config C2] [--frames 20] [--reps 40]"""
import argparse
import os
import statistics as stx
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--warm-s", type=float, default=1.0, help="seconds of launches before measuring")
    ap.add_argument("--order", default="0s,1s,0p,0s,1s,0p",
                    help="variants measured in this order: rt_set_timing value + s (torch.cuda.synchronize) "
                         "or p (poll the closing event, then synchronize)")
    ap.add_argument("--spin", action="store_true",
                    help="hipSetDeviceFlags(hipDeviceScheduleSpin) before the first GPU call: the host spins on "
                         "completion instead of yielding / sleeping")
    a = ap.parse_args()
    import torch
    if a.spin:  # torch's HIP runtime (same soname), before anything initialises the device
        import ctypes
        rc = ctypes.CDLL("libamdhip64.so.7").hipSetDeviceFlags(1)
        print(f"hipSetDeviceFlags(hipDeviceScheduleSpin) -> {rc}")
    from raytracer_hip import Context, abi, scenes
    sc = scenes.config(a.config)
    W, H, F = sc.width, sc.height, a.frames
    buf = torch.empty(F * W * H, dtype=torch.int32, device="cuda")
    ctx = Context(1)
    ctx.set_scene(sc)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream

    def launch():
        ctx.render_bands_batch(W, H, H, 0, 1, F, buf.data_ptr(), W * H * 4, abi.RT_BANDS_INT32, sp)

    t_w = time.perf_counter()
    while time.perf_counter() - t_w < a.warm_s:  # clock ramp
        launch()
        torch.cuda.synchronize()
    for var in a.order.split(","):
        timing, poll = int(var[:-1]), var[-1] == "p"
        ctx.set_timing(timing)
        ctx.reset_stats()
        rows = []
        for _ in range(a.reps):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev0.record(st)
            t1 = time.perf_counter()
            launch()
            t2 = time.perf_counter()
            ev1.record(st)
            t3 = time.perf_counter()
            if poll:
                while not ev1.query():
                    pass
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0, ev0.elapsed_time(ev1) / 1e3))
        s = ctx.stats()
        kern = s["kernel_ms"] / max(1, s["timed_launches"] if "timed_launches" in s else s["launches"]) \
            if s.get("kernel_ms") else float("nan")
        med = [stx.median(c) * 1e6 for c in zip(*rows)]
        print(f"{a.config} F={F} timing={timing} wait={'poll' if poll else 'sync'}: ev0.record {med[0]:.1f} | launch call {med[1]:.1f} | "
              f"ev1.record {med[2]:.1f} | sync wait {med[3]:.1f} | wall {med[4]:.1f} us | ev0->ev1 {med[5]:.1f} us"
              + (f" | kernel (launch events) {kern * 1e3:.1f} us" if timing else ""))
    # the floor: an empty region
    rows = []
    for _ in range(a.reps):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(st)
        ev1.record(st)
        torch.cuda.synchronize()
        rows.append(time.perf_counter() - t0)
    print(f"empty region (two event records + sync{', spin' if a.spin else ''}): wall {stx.median(rows) * 1e6:.1f} us")


if __name__ == "__main__":
    main()
