"""Tick() hand-off under a trace: where each D2H copy of the double-buffered Tick waits.

    cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
        -d $GRAFT_REPO_ROOT/gpurun_out/tick_trace -o tick -- python3 $GRAFT_REPO_ROOT/tools/tick_trace.py

Phases are separated by 200 ms idle gaps; each phase's host window (CLOCK_MONOTONIC ns, the clock
rocprofv3 stamps records with) is printed so that tools/tick_trace_summary.py can cut the trace.
Beside our entry points the same pattern runs on torch alone (a fill kernel on one stream, a D2H
copy on another ordered by an event), into registered and into hipHostMalloc'd memory, so that a
slow case can be put on the runtime's copy path or on ours.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def now():
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def main():
    import torch
    from raytracer_hip import Context, scenes
    sc = scenes.config("C2")
    W, H, n = sc.width, sc.height, 20
    ctx = Context(1)
    ctx.set_scene(sc)
    reg = [np.empty(W * H, dtype=np.int32) for _ in range(2)]
    for hb in reg:
        hb.fill(0)
        ctx.register_host(hb)
    pinned = [torch.empty(W * H, dtype=torch.int32, pin_memory=True) for _ in range(2)]
    pin_np = [p.numpy() for p in pinned]

    def phase(name, fn):
        fn(2)
        time.sleep(0.2)
        t0 = now()
        fn(n)
        t1 = now()
        dt = (t1 - t0) / 1e9 / n
        print(f"PHASE {name:44s} {t0} {t1} {dt * 1e6:8.1f} us/frame {1 / dt:8.0f} fps", flush=True)
        time.sleep(0.2)

    def sync(bufs):
        def f(m):
            for k in range(m):
                ctx.render(W, H, bufs[k % 2])
        return f

    def asy(bufs, every):
        def f(m):
            for k in range(m):
                ctx.render_async(W, H, bufs[k % 2])
                if every and (k + 1) % every == 0:
                    ctx.wait()
            ctx.wait()
        return f

    phase("sync registered", sync(reg))
    phase("async pair registered", asy(reg, 2))
    phase("async deep registered", asy(reg, 0))
    phase("sync hostmalloc", sync(pin_np))
    phase("async pair hostmalloc", asy(pin_np, 2))
    phase("async deep hostmalloc", asy(pin_np, 0))

    # torch alone: kernel on stream A, event, D2H on stream B
    src = [torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in range(2)]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    reg_t = [torch.from_numpy(a) for a in reg]

    def torch2(dst, every):
        def f(m):
            for k in range(m):
                with torch.cuda.stream(sa):
                    src[k % 2].fill_(k)
                    ev = torch.cuda.Event()
                    ev.record(sa)
                sb.wait_event(ev)
                with torch.cuda.stream(sb):
                    dst[k % 2].copy_(src[k % 2], non_blocking=True)
                if every and (k + 1) % every == 0:
                    sb.synchronize()
            torch.cuda.synchronize()
        return f

    def torch1(dst):
        def f(m):
            for k in range(m):
                with torch.cuda.stream(sa):
                    src[k % 2].fill_(k)
                    dst[k % 2].copy_(src[k % 2], non_blocking=True)
            torch.cuda.synchronize()
        return f

    phase("torch 2-stream pair registered", torch2(reg_t, 2))
    phase("torch 2-stream deep registered", torch2(reg_t, 0))
    phase("torch 2-stream deep hostmalloc", torch2(pinned, 0))
    phase("torch 1-stream deep registered", torch1(reg_t))
    phase("torch 1-stream deep hostmalloc", torch1(pinned))
    for hb in reg:
        ctx.unregister_host(hb)


if __name__ == "__main__":
    main()
