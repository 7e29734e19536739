"""Interleaved timing of several builds of libraytracer_hip in ONE process (guide rule 24).

    python tools/ab.py LIB_A LIB_B [LIB_C ...] [--config C2] [--rounds 10] [--frames 50]

Each round renders `frames` frames with every build (order rotating per round); the
library's own HIP-event kernel times are compared (median and min per frame)."""
import argparse
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--strip", default="", help="comma list of spheres,planes,lights,mirrors to remove")
    ap.add_argument("--limit", type=int, default=None, help="override the recursion limit")
    a = ap.parse_args()
    import torch
    from raytracer_hip import abi, scenes
    torch.cuda.set_device(0)
    sc = scenes.config(a.config)
    for what in filter(None, a.strip.split(",")):
        if what == "mirrors":
            sc.spheres = [x for x in sc.spheres if not any(x.material.km)]
        else:
            setattr(sc, what, [])
    if a.limit is not None:
        sc.recursion_limit = a.limit
    W, H = sc.width, sc.height
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    ctxs, libs = [], []
    for path in a.libs:
        lib = abi.load_library(os.path.abspath(path), local=True)
        ctx = C.c_void_p()
        assert lib.rt_create(1, C.byref(ctx)) == 0, lib.rt_last_error(None)
        S, P, L = sc.c_arrays()
        assert lib.rt_set_scene(ctx, S, len(sc.spheres), P, len(sc.planes), L, len(sc.lights),
                                abi.rt_vec3(*sc.ambient), sc.recursion_limit) == 0
        assert lib.rt_set_camera(ctx, C.byref(sc.c_camera())) == 0
        if hasattr(lib, "rt_set_timing"):
            lib.rt_set_timing.argtypes = [C.c_void_p, C.c_int]
            assert lib.rt_set_timing(ctx, 1) == 0  # time every launch
        libs.append(lib)
        ctxs.append(ctx)
    nl = len(libs)
    frames = {i: [] for i in range(nl)}
    crcs = {}
    import zlib
    for rnd in range(a.rounds + 1):
        order = [(rnd + j) % nl for j in range(nl)]
        for i in order:
            lib, ctx = libs[i], ctxs[i]
            lib.rt_reset_stats(ctx)
            for _ in range(a.frames):
                assert lib.rt_render_device(ctx, W, H, C.c_void_p(out.data_ptr()), None) == 0
            st = abi.rt_stats()
            lib.rt_get_stats(ctx, C.byref(st))
            if rnd > 0:  # round 0 = warm-up
                frames[i].append(st.kernel_ms / st.launches)
            crcs[i] = zlib.crc32(out.cpu().numpy().tobytes())
    for i in range(nl):
        v = frames[i]
        print(f"{os.path.basename(a.libs[i]):32s} {a.config}: median {statistics.median(v)*1e3:8.2f} us  "
              f"min {min(v)*1e3:8.2f} us  crc {crcs[i]:08x}")
    for i in range(1, nl):
        print(f"{os.path.basename(a.libs[i])}/A median ratio {statistics.median(frames[i]) / statistics.median(frames[0]):.3f}")


if __name__ == "__main__":
    main()
