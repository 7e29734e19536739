"""Shadow-culling statistics of RT_CULLSTATS builds (experiments): candidate tests per
shadow bundle vs the brute-force S per bundle.
    python tools/cullstats.py BASE_LIB ITER_LIB BUNDLE_LIB --config C4"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=3)
    ap.add_argument("--config", default="C4")
    a = ap.parse_args()
    import torch
    from raytracer_hip import abi, scenes
    sc = scenes.config(a.config)
    W, H = sc.width, sc.height
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    vals = []
    for path in a.libs:
        lib = abi.load_library(os.path.abspath(path), local=True)
        ctx = C.c_void_p()
        assert lib.rt_create(1, C.byref(ctx)) == 0
        S, P, L = sc.c_arrays()
        assert lib.rt_set_scene(ctx, S, len(sc.spheres), P, len(sc.planes), L, len(sc.lights),
                                abi.rt_vec3(*sc.ambient), sc.recursion_limit) == 0
        assert lib.rt_set_camera(ctx, C.byref(sc.c_camera())) == 0
        lib.rt_reset_stats(ctx)
        assert lib.rt_render_device(ctx, W, H, C.c_void_p(out.data_ptr()), None) == 0
        st = abi.rt_stats()
        lib.rt_get_stats(ctx, C.byref(st))
        vals.append(st.shadow_rays)
        lib.rt_destroy(ctx)
    rays, iters, bundles = vals
    S = len(sc.spheres)
    print(f"{a.config}: shadow rays {rays}, bundles {bundles} ({rays / max(bundles, 1):.1f} rays/bundle), "
          f"wave exact-test iterations {iters} = {iters / max(bundles, 1):.2f} per bundle of {S} spheres "
          f"({iters / max(bundles, 1) / S:.3f} of brute force)")


if __name__ == "__main__":
    main()
