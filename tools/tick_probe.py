"""Tick() hand-off probe: where the double-buffered Tick's time goes (C2 1920x1080, 20 frames each).
    python tools/tick_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    import torch
    from raytracer_hip import Context, scenes
    sc = scenes.config("C2")
    W, H, n = sc.width, sc.height, 20
    ctx = Context(1)
    ctx.set_scene(sc)
    hosts = [np.empty(W * H, dtype=np.int32) for _ in range(2)]
    for hb in hosts:
        ctx.register_host(hb)

    def rate(name, fn):
        fn(2)
        t = time.perf_counter()
        fn(n)
        dt = (time.perf_counter() - t) / n
        print(f"{name:48s} {dt * 1e6:8.1f} us/frame  {1 / dt:8.0f} fps", flush=True)

    rate("sync rt_render, one buffer", lambda m: [ctx.render(W, H, hosts[0]) for _ in range(m)])
    rate("sync rt_render, alternating buffers", lambda m: [ctx.render(W, H, hosts[k % 2]) for k in range(m)])

    def asy(m, every, alt):
        for k in range(m):
            ctx.render_async(W, H, hosts[k % 2 if alt else 0])
            if every and (k + 1) % every == 0:
                ctx.wait()
        ctx.wait()
    rate("async, alternating buffers, one wait", lambda m: asy(m, 0, True))
    rate("async, one buffer, one wait", lambda m: asy(m, 0, False))
    rate("async, alternating, wait every frame", lambda m: asy(m, 1, True))
    rate("async, alternating, wait every 2 frames", lambda m: asy(m, 2, True))
    # the same deep queue into hipHostMalloc'd memory (torch pinned tensors) instead of registered memory
    pinned = [torch.empty(W * H, dtype=torch.int32, pin_memory=True) for _ in range(2)]

    def asy_pinned(m):
        for k in range(m):
            ctx.lib.rt_render_async(ctx.ptr, W, H, pinned[k % 2].data_ptr())
        ctx.wait()
    rate("async into hipHostMalloc memory, one wait", asy_pinned)
    # the bare copy: 8.3 MB device -> pinned host through torch
    src = torch.empty(W * H, dtype=torch.int32, device="cuda")
    dst = torch.empty(W * H, dtype=torch.int32, pin_memory=True)

    def cp(m):
        for _ in range(m):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
    rate("torch D2H 8.3 MB into pinned memory", cp)
    for hb in hosts:
        ctx.unregister_host(hb)


if __name__ == "__main__":
    main()
