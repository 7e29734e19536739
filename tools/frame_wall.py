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
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(a.inflight - 1)]
    sp = [s.cuda_stream for s in streams]
    for k in range(20):
        ctx.render_device(W, H, outs[k % a.inflight].data_ptr(), sp[k % a.inflight])
    torch.cuda.synchronize()
    res, enq = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        for k in range(a.frames):
            ctx.render_device(W, H, outs[k % a.inflight].data_ptr(), sp[k % a.inflight])
        enq.append((time.perf_counter() - t0) / a.frames * 1e6)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / a.frames * 1e6)
    st = ctx.stats()
    kern = st["kernel_ms"] / st["launches"] * 1e3 if st["kernel_ms"] else float("nan")
    print(f"{os.path.basename(a.lib) or 'in-tree'} {a.config} {W}x{H} strip={a.strip or '-'} inflight={a.inflight}: "
          f"wall/frame min {min(res):.2f} us median {sorted(res)[len(res)//2]:.2f} us; host enqueue/frame {min(enq):.2f} us")


if __name__ == "__main__":
    main()
