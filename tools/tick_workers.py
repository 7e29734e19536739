#!/usr/bin/env python3
"""Tick() rates of the plugin path (rt_render / rt_render_async into registered host buffers) per config,
band-worker count and chunk count -- the PCIe hand-off of DESIGN §1e measured on one box.
    python tools/tick_workers.py --configs C2,C5 --worlds 1,2 [--shared] [--chunks 1,2,4] [--frames 20]
--shared puts the workers on one device (RT_CREATE_SHARED_DEVICE): the code path of n devices, but one
PCIe link, so rates at n > 1 say nothing about a real node."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C5")
    ap.add_argument("--worlds", default="1")
    ap.add_argument("--chunks", default="", help="comma list of RT_TICK_CHUNKS values ('' = the default)")
    ap.add_argument("--shared", action="store_true")
    ap.add_argument("--copy", default="", help="RT_TICK_COPY for the run: runtime | kernel ('' = the library's default)")
    ap.add_argument("--async-copy", default="", help="RT_TICK_ASYNC for the run: stream | slice ('' = default)")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    from raytracer_hip import Context, abi, scenes
    if a.copy:
        os.environ["RT_TICK_COPY"] = a.copy
    if a.async_copy:
        os.environ["RT_TICK_ASYNC"] = a.async_copy
    for cid in a.configs.split(","):
        sc = scenes.config(cid)
        W, H = sc.width, sc.height
        for world in map(int, a.worlds.split(",")):
            ctx = Context(world, abi.RT_CREATE_SHARED_DEVICE if a.shared else 0)
            ctx.set_scene(sc)
            bufs = [np.zeros(W * H, dtype=np.int32) for _ in range(2)]
            for b in bufs:
                ctx.register_host(b)
            for ch in (a.chunks.split(",") if a.chunks else [""]):
                if ch:
                    os.environ["RT_TICK_CHUNKS"] = ch
                else:
                    os.environ.pop("RT_TICK_CHUNKS", None)

                def sync():
                    for _ in range(a.frames):
                        ctx.render(W, H, bufs[0])

                def pair():
                    for k in range(a.frames):
                        ctx.render_async(W, H, bufs[k % 2])
                        if k % 2:
                            ctx.wait()
                    ctx.wait()
                out = []
                for name, fn in (("sync", sync), ("async", pair)):
                    fn()
                    rates = []
                    for _ in range(a.reps):
                        t = time.perf_counter()
                        fn()
                        rates.append(a.frames / (time.perf_counter() - t))
                    r = sorted(rates)[len(rates) // 2]
                    out.append(f"{name} {r:8.1f} fps ({W * H * 4 * r / 1e9:6.1f} GB/s of frame)")
                print(f"{cid} world {world}{' shared' if a.shared else ''} copy {a.copy or 'default'}/{a.async_copy or 'default'} chunks "
                      f"{ch or 'default'}: " + "; ".join(out),
                      flush=True)
            for b in bufs:
                ctx.unregister_host(b)
            ctx.close()


if __name__ == "__main__":
    main()
