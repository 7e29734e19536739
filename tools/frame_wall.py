"""Wall-clock per frame of back-to-back rt_render_device calls (bench.py's timed loop
without the rest), to separate kernel time from per-frame gaps.
    python tools/frame_wall.py [--config C2] [--frames 400]"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--strip", default="", help="comma list of spheres,planes,lights to remove")
    ap.add_argument("--size", default="", help="WxH override")
    ap.add_argument("--inflight", type=int, default=1, help="frames in flight (streams/buffers)")
    ap.add_argument("--lib", default="", help="library build to load instead of the in-tree one")
    ap.add_argument("--bands", default="", help="R/N: trace only rank R's 8-row bands of an N-rank world")
    ap.add_argument("--batch", type=int, default=1, help="frames per launch (rt_render_bands_batch)")
    ap.add_argument("--no-count", action="store_true", help="rt_set_counting(0): the launches count no rays")
    a = ap.parse_args()
    import torch
    from raytracer_hip import Context, abi, scenes
    if a.lib:
        abi.LIB_PATH = os.path.abspath(a.lib)
    sc = scenes.config(a.config)
    for what in filter(None, a.strip.split(",")):
        setattr(sc, what, [])
    if a.size:
        sc = sc.resized(*map(int, a.size.split("x")))
    W, H = sc.width, sc.height
    outs = [torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in range(a.inflight)]
    ctx = Context(1)
    ctx.set_scene(sc)
    if a.no_count:
        ctx.set_counting(False)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(a.inflight - 1)]
    sp = [s.cuda_stream for s in streams]
    ptrs = [o.data_ptr() for o in outs]
    if a.batch > 1:
        R, N = map(int, (a.bands or "0/1").split("/"))
        big = [torch.empty(a.batch * W * H, dtype=torch.int32, device="cuda") for _ in range(a.inflight)]
        bptr = [b.data_ptr() for b in big]
        a.frames = a.frames // a.batch * a.batch

        def frame(k):  # one launch per a.batch frames
            if k % a.batch == 0:
                i = (k // a.batch) % a.inflight
                ctx.render_bands_batch(W, H, 8, R, N, a.batch, bptr[i], W * H * 4, abi.RT_BANDS_FRAME, sp[i])
    elif a.bands:
        R, N = map(int, a.bands.split("/"))

        def frame(k):
            ctx.render_bands_ex(W, H, 8, R, N, ptrs[k % a.inflight], abi.RT_BANDS_INT32, sp[k % a.inflight])
    else:
        def frame(k):
            ctx.render_device(W, H, ptrs[k % a.inflight], sp[k % a.inflight])
    for k in range(20):
        frame(k)
    torch.cuda.synchronize()
    res, enq = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        for k in range(a.frames):
            frame(k)
        enq.append((time.perf_counter() - t0) / a.frames * 1e6)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / a.frames * 1e6)
    st = ctx.stats()
    kern = st["kernel_ms"] / st["launches"] * 1e3 if st["kernel_ms"] else float("nan")
    order = ctx.dispatch_order() if hasattr(ctx, "dispatch_order") else None
    print(f"{os.path.basename(a.lib) or 'in-tree'} {a.config} {W}x{H} strip={a.strip or '-'} bands={a.bands or '-'} batch={a.batch} inflight={a.inflight}{' no-count' if a.no_count else ''}: "
          f"wall/frame min {min(res):.2f} us median {sorted(res)[len(res)//2]:.2f} us; host enqueue/frame {min(enq):.2f} us"
          + (f"; dispatch order {order}" if order is not None else ""))


if __name__ == "__main__":
    main()
