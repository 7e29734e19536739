"""Wall per frame of a scene with general specular exponents (the direct kernel's GPOW instantiation):
C3 with its plastic and metal spheres at n = 3.7 / 7.25, one frame per launch into HBM, median of 5 runs of 200.
    python tools/probes/gpow_wall.py [--lib path.so]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    if a.lib:
        from raytracer_hip import abi
        abi.LIB_PATH = os.path.abspath(a.lib)
    import torch
    from raytracer_hip import Context, scenes
    sc = scenes.config("C3")
    sph = []
    for i, s in enumerate(sc.spheres):
        m = s.material
        if any(m.ks):
            m = scenes.Material(m.kd, m.ka, m.ks, scenes.f32(3.7 if i % 2 else 7.25), m.km)
        sph.append(scenes.Sphere(s.center, s.radius, m))
    sc = scenes.Scene("C3gpow", sc.width, sc.height, sph, sc.planes, sc.lights, sc.ambient, sc.recursion_limit, sc.camera)
    W, H = sc.width, sc.height
    with Context(1) as ctx:
        ctx.set_scene(sc)
        ctx.set_counting(False)
        dev = torch.empty(W * H, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        rates = []
        for rep in range(6):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(200):
                ctx.render_device(W, H, dev.data_ptr(), st)
            torch.cuda.synchronize()
            if rep:
                rates.append((time.perf_counter() - t) / 200 * 1e6)
        print(f"{os.path.basename(a.lib) or 'in-tree'} C3 with n = 3.7 / 7.25: {sorted(rates)[2]:.2f} us per lone frame "
              f"(runs {[round(r, 2) for r in rates]})", flush=True)


if __name__ == "__main__":
    main()
