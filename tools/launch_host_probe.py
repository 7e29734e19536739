"""Host time of one trace launch call (ctypes -> C ABI -> hipLaunchKernel), per entry point, C2 1080p,
20 frames per launch: rt_render_bands_batch (N = 1 bench), rt_render_bands_tiles (N > 1 ranks, fused
encoder), rt_finish_wire, rt_decode_gathered.  Each call timed alone after a device synchronisation."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    import torch
    from raytracer_hip import Context, abi, scenes, wire_layout
    sc = scenes.config("C2")
    W, H, F = sc.width, sc.height, 20
    ctx = Context(1)
    ctx.set_scene(sc)
    s = torch.cuda.current_stream().cuda_stream
    out = torch.empty(F * W * H, dtype=torch.int32, device="cuda")
    lay = wire_layout(W, H, 8, 1, F)
    wire = torch.empty(int(lay.max_bytes) + 256, dtype=torch.uint8, device="cuda")
    size = torch.zeros(1, dtype=torch.int64, device="cuda")
    frames = torch.empty(F * W * H, dtype=torch.int32, device="cuda")

    def t(fn, n=30):
        xs = []
        for _ in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            xs.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        return statistics.median(xs) * 1e6, min(xs) * 1e6

    calls = {
        "render_bands_batch (20 frames)": lambda: ctx.render_bands_batch(W, H, H, 0, 1, F, out.data_ptr(), W * H * 4,
                                                                          abi.RT_BANDS_INT32, s),
        "render_bands_tiles (20 frames)": lambda: ctx.render_bands_tiles(W, H, 8, 0, 1, 0, F, F, wire.data_ptr(), s),
        "finish_wire": lambda: ctx.finish_wire(W, H, 8, 0, 1, F, wire.data_ptr(), size.data_ptr(), s),
        "decode_gathered": lambda: ctx.decode_gathered(W, H, 8, 1, wire.data_ptr(), int(lay.max_bytes + 255) // 256 * 256,
                                                       F, frames.data_ptr(), W * H, s, first_rank=0),
        "torch empty kernel (fill_)": lambda: size.fill_(0),
    }
    for name, fn in calls.items():
        med, mn = t(fn)
        print(f"{name:36s} host us per call: median {med:7.1f}  min {mn:7.1f}", flush=True)


if __name__ == "__main__":
    main()
