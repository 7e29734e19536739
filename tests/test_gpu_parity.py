"""GPU parity: libraytracer_hip (HIP, gfx950) against the CPU oracle, bit-exact int32 pixels
and identical ray counts.  Every call goes through the C ABI.

Bar: bit-exact for every pixel (integer packing of float colours whose computation is
restated operation by operation) and identical visible-path ray counts.
"""
import zlib

import numpy as np
import pytest

from raytracer_hip import Context, RayTracer, Surface, abi, bands_of, scenes

pytestmark = pytest.mark.gpu


def crc(a):
    return f"{zlib.crc32(np.ascontiguousarray(a, dtype=np.int32).tobytes()) & 0xFFFFFFFF:08x}"


def ray_counts(st):
    return {k: st[k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


def render_gpu(ctx, sc):
    ctx.set_scene(sc)
    ctx.reset_stats()
    px = ctx.render(sc.width, sc.height).copy()
    return px, ctx.stats()


def assert_same(px, want, what):
    bad = px != want
    if bad.any():
        ys, xs = np.nonzero(bad)
        pytest.fail(f"{what}: {int(bad.sum())} of {bad.size} pixels differ; first at (x={xs[0]}, y={ys[0]}): "
                    f"gpu {px[ys[0], xs[0]]:#08x} oracle {want[ys[0], xs[0]]:#08x}")


@pytest.mark.parametrize("cid", ["REF_64", "REF_128", "C1_64", "C2_96x54", "C3_96x54", "C4_64x36"])
def test_small_frames_vs_committed_golden(gpu_ctx, golden, cid):
    import os
    e = golden["cases"][cid]
    sc = scenes.config(e["config"]).resized(e["width"], e["height"])
    px, st = render_gpu(gpu_ctx, sc)
    want = np.load(os.path.join(os.path.dirname(__file__), "golden", e["frame"]))
    assert_same(px, want, cid)
    assert ray_counts(st) == {k: e["stats"][k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


@pytest.mark.parametrize("cid", ["REF_512", "REF_1280x720", "C1", "C2", "C3", "C4", "C5"])
def test_full_size_frames_vs_golden_and_oracle(gpu_ctx, golden, oracle, cid):
    """BASELINE.json configs at their full sizes (C5 = 7680x4320, 33 Mpixel)."""
    e = golden["cases"][cid]
    sc = scenes.config(e["config"]).resized(e["width"], e["height"])
    px, st = render_gpu(gpu_ctx, sc)
    if crc(px) != e["crc32"]:
        want, _ = oracle.render(sc, oracle.MODE_NEAREST)
        assert_same(px, want, cid)
    assert ray_counts(st) == {k: e["stats"][k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}
    assert st["pixels"] == e["width"] * e["height"]


@pytest.mark.parametrize("seed", list(range(40)))
def test_random_scenes_vs_oracle(gpu_ctx, oracle, seed):
    import random_scenes
    sc = random_scenes.random_scene(seed)
    px, st = render_gpu(gpu_ctx, sc)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 4)
    ref, _ = oracle.render(sc, oracle.MODE_REFERENCE, 4)
    assert np.array_equal(want, ref)
    assert_same(px, want, sc.name)
    assert ray_counts(st) == {k: ost[k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


@pytest.mark.parametrize("seed", list(range(100, 130)))
def test_dense_random_scenes_vs_oracle(gpu_ctx, oracle, seed):
    """12-100 spheres: the wave-bundle culling path, 64-sphere mask chunks."""
    import random_scenes
    sc = random_scenes.random_scene(seed, 128, 96, dense=True)
    px, st = render_gpu(gpu_ctx, sc)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 4)
    assert_same(px, want, sc.name)
    assert ray_counts(st) == {k: ost[k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


@pytest.mark.parametrize("n_lights", [1, 4, 5, 8])
@pytest.mark.parametrize("limit", [0, 5, 7, 9])
def test_bundle_light_counts_and_stacks(gpu_ctx, oracle, n_lights, limit):
    """The bundle kernel on either side of the merged shadow pass's bound (L <= 4 lights: one loop
    over the union of the lights' candidates; L = 5, 8: a pass per light) and across its stacks
    (limit 0 / 5 / 7: the LDS stack with K = 1 / 6 / 8; limit 9: the scratch stack), with mirror
    chains: every pixel and ray count against the oracle."""
    import random_scenes
    base = random_scenes.random_scene(100 + 7 * n_lights + limit, 128, 96, dense=True)
    rng = np.random.default_rng(1000 * n_lights + limit)
    lights = [scenes.Light(tuple(float(np.float32(x)) for x in rng.uniform(-30, 30, 3)),
                           float(np.float32(rng.uniform(0.2, 1.2)))) for _ in range(n_lights)]
    sc = scenes.Scene(f"bundle_L{n_lights}_lim{limit}", 128, 96, base.spheres, base.planes, lights, base.ambient,
                      limit, base.camera)
    px, st = render_gpu(gpu_ctx, sc)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 8)
    assert_same(px, want, sc.name)
    assert ray_counts(st) == {k: ost[k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


def shadow_grid_scene(seed, width=160, height=96):
    """A C4-like scene for the merged shadow pass's per-light grids (12-64 spheres, 1-4 lights):
    mirror-heavy materials (deep fold levels, scattered hit points), coordinates at unit, 30x and
    1000x scale (the grid's lane bound and margins scale with the scene), grazing lights, ground
    and back planes reaching far beyond the bound, and cameras anywhere in the scene."""
    rng = np.random.default_rng(20_000 + seed)
    scale = [1.0, 30.0, 1000.0][seed % 3]
    f = lambda x: float(np.float32(x))  # noqa: E731
    ns = int(rng.integers(12, 65))
    mats = [scenes.Material.mirror(scenes.ONE), scenes.Material.diffuse((0.8, 0.3, 0.2)),
            scenes.Material.plastic((0.2, 0.7, 0.3), 2.0), scenes.Material.diffuse_mirror((0.6, 0.6, 0.9), (0.5,) * 3)]
    sph = [scenes.Sphere((f(rng.uniform(-8, 8) * scale), f(rng.uniform(-0.7, 1.0) * scale), f(rng.uniform(4, 32) * scale)),
                         f(rng.uniform(0.25, 1.0) * scale), mats[int(rng.integers(0, 4))]) for _ in range(ns)]
    if seed % 4 == 1:
        sph[3] = scenes.Sphere(sph[3].center, f(1e-3 * scale), mats[1])  # tiny
    planes = [scenes.Plane((0.0, f(-1 * scale), 0.0), (0.0, 1.0, 0.0), scenes.REF_PLANES[0].material),
              scenes.Plane((0.0, 0.0, f(48 * scale)), (0.0, 0.0, -1.0), scenes.Material.diffuse((0.6, 0.6, 0.6)))]
    nl = int(rng.integers(1, 5))
    lights = [scenes.Light((f(rng.uniform(-40, 40) * scale), f(rng.uniform(0.5, 15) * scale),
                            f(rng.uniform(-10, 40) * scale)), 1.0) for _ in range(nl)]
    if seed % 5 == 2:
        lights[0] = scenes.Light((f(33 * scale), f(1e-3), f(10 * scale)), 1.0)  # grazing
    cam = ((f(rng.uniform(-3, 3) * scale), f(rng.uniform(-0.5, 2) * scale), f(rng.uniform(-4, 10) * scale)),
           f(rng.uniform(-0.8, 0.8)), f(rng.uniform(-0.3, 0.5)))
    return scenes.Scene(f"grid{seed}", width, height, sph, planes, lights, scenes.REF_AMBIENT,
                        int(rng.choice([1, 3, 5, 7])), cam)


@pytest.mark.parametrize("seed", list(range(30)))
def test_shadow_grid_scenes_vs_oracle(gpu_ctx, oracle, seed, monkeypatch):
    """The bundle kernel's merged shadow pass takes each lane's sphere candidates from per-light
    grids (rt_api.cpp build_shadow_grid); RT_SHADOW_GRID=0 at rt_set_scene keeps the per-level
    bound instead.  Both must give the oracle's pixels and ray counts."""
    sc = shadow_grid_scene(seed)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 8)
    for grid in ("1", "0"):
        monkeypatch.setenv("RT_SHADOW_GRID", grid)
        px, st = render_gpu(gpu_ctx, sc)
        assert_same(px, want, f"{sc.name} RT_SHADOW_GRID={grid}")
        assert ray_counts(st) == ray_counts(ost)


@pytest.mark.parametrize("seed", list(range(24)))
def test_trace_cluster_precull_vs_oracle(gpu_ctx, oracle, seed, monkeypatch):
    """The bundle kernel's per-lane cluster pre-cull of trace bundles too wide for the bundle cull (rt_kernel.hip
    cluster_mask; clusters of RT_TRACE_CLUSTERS spheres built at rt_set_scene, 0 = off): the mirror-heavy grid
    scenes at unit, 30x and 1000x scale, clusters of 4, 2 and 8 (the default) spheres and none -- every pixel
    and ray count the oracle's."""
    sc = shadow_grid_scene(1000 + seed, 128, 80)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 8)
    for z in ("4", "2", "8", "0"):
        monkeypatch.setenv("RT_TRACE_CLUSTERS", z)
        px, st = render_gpu(gpu_ctx, sc)
        assert_same(px, want, f"{sc.name} RT_TRACE_CLUSTERS={z}")
        assert ray_counts(st) == ray_counts(ost)


def shadow_pre_scene(seed, width=160, height=96):
    """A C2/C3-like scene for the direct kernel's per-lane shadow pre-test (1-11 spheres, 1-4 lights): diffuse,
    plastic and mirror spheres at 1e-3x, unit, 30x and 1000x scale, lights that graze the floor, sit at the
    origin (2a = 0: the literal root formula, no pre-test), have a = p.p below 2^-40 (no culling) or lie far out,
    a tiny sphere and one far from the others, a checkered floor and cameras anywhere in the scene."""
    rng = np.random.default_rng(30_000 + seed)
    scale = [1.0, 30.0, 1000.0, 1e-3][seed % 4]
    f = lambda x: float(np.float32(x))  # noqa: E731
    ns = int(rng.integers(1, 12))
    mats = [scenes.Material.mirror(scenes.ONE), scenes.Material.diffuse((0.8, 0.3, 0.2)),
            scenes.Material.plastic((0.2, 0.7, 0.3), 1.0), scenes.Material.diffuse_mirror((0.6, 0.6, 0.9), (0.5,) * 3),
            scenes.Material.plastic((0.9, 0.9, 0.2), 0.5)]
    sph = [scenes.Sphere((f(rng.uniform(-6, 6) * scale), f(rng.uniform(-0.7, 1.5) * scale), f(rng.uniform(3, 20) * scale)),
                         f(rng.uniform(0.3, 1.5) * scale), mats[int(rng.integers(0, 5))]) for _ in range(ns)]
    if seed % 5 == 1 and ns > 1:
        sph[1] = scenes.Sphere(sph[1].center, f(1e-3 * scale), mats[1])  # tiny
    if seed % 7 == 3 and ns > 2:
        sph[2] = scenes.Sphere((f(4e4 * scale), 0.0, f(9 * scale)), f(scale), mats[2])  # far from the others
    planes = [scenes.Plane((0.0, f(-1 * scale), 0.0), (0.0, 1.0, 0.0), scenes.REF_PLANES[0].material)]
    nl = int(rng.integers(1, 5))
    lights = [scenes.Light((f(rng.uniform(-30, 30) * scale), f(rng.uniform(0.5, 12) * scale),
                            f(rng.uniform(-10, 30) * scale)), 1.0) for _ in range(nl)]
    if seed % 3 == 0:
        lights[0] = scenes.Light((f(25 * scale), f(1e-3 * scale), f(8 * scale)), 1.0)  # grazing
    if seed % 6 == 1:
        lights[-1] = scenes.Light((0.0, 0.0, 0.0), 0.7)  # 2a = 0
    if seed % 8 == 5:
        lights[-1] = scenes.Light((f(1e-25), 0.0, 0.0), 0.7)  # a < 2^-40
    cam = ((f(rng.uniform(-2, 2) * scale), f(rng.uniform(-0.5, 2) * scale), f(rng.uniform(-4, 2) * scale)),
           f(rng.uniform(-0.6, 0.6)), f(rng.uniform(-0.3, 0.4)))
    return scenes.Scene(f"pre{seed}", width, height, sph, planes, lights, scenes.REF_AMBIENT,
                        int(rng.choice([0, 1, 2, 4])), cam)


@pytest.mark.parametrize("seed", list(range(32)))
def test_direct_shadow_pretest_vs_oracle(gpu_ctx, oracle, seed, monkeypatch):
    """The direct kernel's per-lane shadow pre-test (rt_kernel.hip shadow_pre_keep, records built at
    rt_set_scene; RT_SHADOW_PRE=0 = every sphere tested): both give the oracle's pixels and ray counts."""
    sc = shadow_pre_scene(seed)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 8)
    for pre in ("1", "0"):
        monkeypatch.setenv("RT_SHADOW_PRE", pre)
        px, st = render_gpu(gpu_ctx, sc)
        assert_same(px, want, f"{sc.name} RT_SHADOW_PRE={pre}")
        assert ray_counts(st) == ray_counts(ost)


POW_EXPONENTS = [3.7, 7.25, 12.0, float.fromhex("0x1.946b02p+4"), float.fromhex("0x1.273c82p+2"), 2.486319, 21.299271, 60.566631, 9.88111, 0.75, 1.5,
                 33.0, 0.1, 5.0e-3, 63.9]


@pytest.mark.parametrize("k", list(range(len(POW_EXPONENTS))))
def test_generic_specular_exponents_vs_oracle(gpu_ctx, oracle, k):
    """Specular exponents other than 0.5, 1, 2 (Math.Pow, RayTracer.cs:691): the kernels run the restatement of
    glibc's pow (csrc/rt_pow.h), the oracle the host's glibc pow.  Metal and Plastic spheres with the exponent,
    among them the two at which the device's own pow and glibc round to different floats (profiles/r06_pow_check.txt),
    on the direct kernel (C3's 8 spheres) and the bundle kernel (C4's 64): every pixel the oracle's."""
    n = float(np.float32(POW_EXPONENTS[k]))
    for cid, size in (("C3", (480, 270)), ("C4", (384, 216))):
        base = scenes.config(cid)
        sph = [scenes.Sphere(s.center, s.radius, (scenes.Material.metal if i % 2 else scenes.Material.plastic)(
            s.material.kd if any(s.material.kd) else (0.7, 0.6, 0.5), n)) if i % 3 != 2 else s
               for i, s in enumerate(base.spheres)]
        pl = [scenes.Plane(p.center, p.normal, scenes.Material.metal((0.8, 0.8, 0.8), n)) for p in base.planes]
        sc = scenes.Scene(f"{cid}_pow{k}", size[0], size[1], sph, pl, base.lights, base.ambient, base.recursion_limit,
                          base.camera)
        px, st = render_gpu(gpu_ctx, sc)
        want, ost = oracle.render(sc, oracle.MODE_NEAREST, 8)
        assert_same(px, want, f"{sc.name} n={n!r}")
        assert ray_counts(st) == ray_counts(ost)


@pytest.mark.parametrize("n_lights", [3000, 4200])
def test_many_lights_with_and_without_the_shadow_cull_table(gpu_ctx, oracle, n_lights):
    """The bundle kernel's shadow culling reads the sphere centres pre-projected into each light's
    frame from a [lights][spheres] table built when lights x spheres <= 65536 (16 spheres: 3000
    lights have one, 4200 do not and trace their shadow rays unculled); both must match."""
    import random_scenes
    base = random_scenes.random_scene(101, 24, 16, dense=True)
    rng = np.random.default_rng(n_lights)
    lights = [scenes.Light(tuple(float(np.float32(x)) for x in rng.uniform(-30, 30, 3)),
                           float(np.float32(rng.uniform(0.0002, 0.0004)))) for _ in range(n_lights)]
    sc = scenes.Scene(f"lights{n_lights}", 24, 16, base.spheres[:16], base.planes, lights, base.ambient, 2,
                      base.camera)
    px, st = render_gpu(gpu_ctx, sc)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 8)
    assert_same(px, want, sc.name)
    assert ray_counts(st) == {k: ost[k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


@pytest.mark.parametrize("seed", list(range(200)))
def test_camera_sweep_vs_oracle(gpu_ctx, oracle, seed):
    """Primary screen boxes (and both kernels' primary paths) under arbitrary views."""
    from random_scenes import camera_sweep_scene
    sc = camera_sweep_scene(seed)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 4)
    px, st = render_gpu(gpu_ctx, sc)
    assert_same(px, want, sc.name)
    assert ray_counts(st) == ray_counts(ost)


@pytest.mark.parametrize("w,h", [(1, 1), (17, 13), (15, 16), (16, 15), (33, 65), (1000, 3)])
def test_ragged_frame_sizes(gpu_ctx, oracle, w, h):
    sc = scenes.config("C3").resized(w, h)
    px, _ = render_gpu(gpu_ctx, sc)
    want, _ = oracle.render(sc, oracle.MODE_NEAREST, 4)
    assert_same(px, want, f"{w}x{h}")


@pytest.mark.parametrize("limit", [0, 1, 2, 3, 4, 7, 8, 9, 32, 63])
def test_recursion_limits_across_stack_variants(gpu_ctx, oracle, limit):
    """K = 1/2/4/8 register stacks and the 64-deep scratch stack (limit+1 records)."""
    sc = scenes.reference(160, 120)
    sc.recursion_limit = limit
    sc.camera = ((-1.5, -0.5, 4.0), -0.9, 0.1)  # looks at the mirror sphere over the mirror floor
    px, st = render_gpu(gpu_ctx, sc)
    want, ost = oracle.render(sc, oracle.MODE_NEAREST, 4)
    assert_same(px, want, f"limit {limit}")
    assert ray_counts(st) == {k: ost[k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


def test_empty_scene_is_black(gpu_ctx):
    sc = scenes.Scene("empty", 40, 30, [], [], [], scenes.REF_AMBIENT, 0)
    px, st = render_gpu(gpu_ctx, sc)
    assert (px == 0).all() and st["reflect_rays"] == 0 and st["shadow_rays"] == 0


def test_no_lights_only_ambient_and_mirrors(gpu_ctx, oracle):
    sc = scenes.reference(64, 64)
    sc.lights = []
    px, st = render_gpu(gpu_ctx, sc)
    want, _ = oracle.render(sc, oracle.MODE_NEAREST, 4)
    assert_same(px, want, "no lights")
    assert st["shadow_rays"] == 0


@pytest.mark.parametrize("band_rows,nranks", [(8, 2), (8, 3), (5, 8), (16, 1), (7, 5), (1, 4)])
def test_row_bands_reassemble(gpu_ctx, band_rows, nranks):
    """rt_render_bands on every band set + rt_scatter_bands == the full frame (the multi-GPU data path)."""
    import torch
    sc = scenes.config("C3").resized(200, 117)
    gpu_ctx.set_scene(sc)
    W, H = sc.width, sc.height
    full = gpu_ctx.render(W, H).copy()
    frame = torch.full((H * W,), -1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for r in range(nranks):
        nb = bands_of(H, band_rows, r, nranks)
        buf = torch.full((max(1, nb) * band_rows * W,), -7, dtype=torch.int32, device="cuda")
        got = gpu_ctx.render_bands(W, H, band_rows, r, nranks, buf.data_ptr(), stream)
        assert got == nb
        gpu_ctx.scatter_bands(W, H, band_rows, r, nranks, buf.data_ptr(), frame.data_ptr(), stream)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().reshape(H, W), full)


def test_render_device_on_torch_stream(gpu_ctx, golden):
    import torch
    e = golden["cases"]["C2"]
    sc = scenes.config("C2")
    gpu_ctx.set_scene(sc)
    out = torch.zeros(sc.width * sc.height, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gpu_ctx.render_device(sc.width, sc.height, out.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert crc(out.cpu().numpy()) == e["crc32"]


@pytest.mark.parametrize("order", [0, 1, 2, 3])
@pytest.mark.parametrize("cid", ["C1", "C2", "C3", "REF_1280x720"])
def test_single_frame_dispatch_orders(golden, monkeypatch, cid, order):
    """Each single-frame dispatch order (rows by estimated cost, bottom to top, rows varying fastest, every
    tile by measured duration: rt_dispatch_order's candidates, fixed through RT_DISPATCH_ORDER) renders the
    golden frame, through rt_render and rt_render_device (order 3: the first launch records the tile
    durations, the later ones run the sorted order)."""
    import torch
    monkeypatch.setenv("RT_DISPATCH_ORDER", str(order))
    e = golden["cases"][cid]
    sc = scenes.config(e["config"]).resized(e["width"], e["height"])
    ctx = Context(1)
    try:
        ctx.set_scene(sc)
        assert ctx.dispatch_order() == order
        for _ in range(2):
            assert crc(ctx.render(sc.width, sc.height)) == e["crc32"]
        out = torch.zeros(sc.width * sc.height, dtype=torch.int32, device="cuda")
        for _ in range(2):
            out.zero_()
            ctx.render_device(sc.width, sc.height, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert crc(out.cpu().numpy()) == e["crc32"]
    finally:
        ctx.close()


@pytest.mark.parametrize("cid,size", [("C3", (203, 117)), ("C3", (8, 8)), ("C3", (9, 300)), ("C3", (1000, 9)),
                                      ("C4", (203, 117)), ("C4", (8, 8)), ("C4", (9, 300))])
def test_measured_tile_order_ragged_vs_oracle(oracle, monkeypatch, size, cid):
    """The measured tile order (candidate 3) on frames whose tile count is not a multiple of the 4-tile
    workgroup and whose edge tiles are partial -- the direct kernel (C3's scene) and the bundle kernel (C4's):
    the padded entries trace nothing, every pixel = the oracle's, on the recording launch and on the sorted
    ones; a size change records again."""
    monkeypatch.setenv("RT_DISPATCH_ORDER", "3")
    sc = scenes.config(cid).resized(*size)
    want, _ = oracle.render(sc, oracle.MODE_NEAREST, 8)
    ctx = Context(1)
    try:
        ctx.set_scene(sc)
        for _ in range(3):
            assert_same(ctx.render(sc.width, sc.height).copy(), want, f"{cid} {size}")
        sc2 = scenes.config(cid).resized(size[1], size[0])
        want2, _ = oracle.render(sc2, oracle.MODE_NEAREST, 8)
        ctx.set_scene(sc2)
        for _ in range(2):
            assert_same(ctx.render(sc2.width, sc2.height).copy(), want2, f"{cid} {size[::-1]}")
    finally:
        ctx.close()


@pytest.mark.parametrize("order", [0, 3, None])
@pytest.mark.parametrize("cid", ["C4", "C5"])
def test_bundle_lone_frame_orders(golden, monkeypatch, cid, order):
    """The bundle kernel's one-frame launches in natural order (0), in the measured tile order (3: the first
    launch records the tile durations) and under the library's own choice: the golden frames, through
    rt_render_device and rt_render."""
    import torch
    if order is None:
        monkeypatch.delenv("RT_DISPATCH_ORDER", raising=False)
    else:
        monkeypatch.setenv("RT_DISPATCH_ORDER", str(order))
    e = golden["cases"][cid]
    sc = scenes.config(cid)
    W, H = sc.width, sc.height
    ctx = Context(1)
    try:
        ctx.set_scene(sc)
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for k in range(60 if order is None else 3):  # (None: well past the tuner's 28 probes and its recording)
            ctx.render_device(W, H, out.data_ptr(), st)
            if k % 10 == 9 or order is not None:
                torch.cuda.synchronize()
                assert crc(out.cpu().numpy()) == e["crc32"]
                out.zero_()
        torch.cuda.synchronize()
        if order is not None:
            assert ctx.dispatch_order() == order
        else:  # (1 and 2 launch the bundle kernel in natural order, like 0)
            assert ctx.dispatch_order() in (0, 1, 2, 3)
        assert crc(ctx.render(W, H)) == e["crc32"]
    finally:
        ctx.close()


def test_dispatch_order_measured_then_kept(golden):
    """Without RT_DISPATCH_ORDER the first single-frame launches of a scene and size time the candidates
    in turn and then keep one; every frame along the way is the golden one, and a new scene (or size)
    measures again."""
    import torch
    ctx = Context(1)
    try:
        for cid in ("C2", "C1"):
            e = golden["cases"][cid]
            sc = scenes.config(e["config"]).resized(e["width"], e["height"])
            ctx.set_scene(sc)
            assert ctx.dispatch_order() == -1
            outs = [torch.zeros(sc.width * sc.height, dtype=torch.int32, device="cuda") for _ in range(3)]
            st = torch.cuda.current_stream().cuda_stream
            for k in range(60):
                ctx.render_device(sc.width, sc.height, outs[k % 3].data_ptr(), st)
                if k % 10 == 9:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            assert ctx.dispatch_order() in (0, 1, 2, 3)
            for o in outs:
                assert crc(o.cpu().numpy()) == e["crc32"]
    finally:
        ctx.close()


@pytest.mark.parametrize("cid", ["C3", "C4"])
def test_measured_tile_order_mixed_streams_and_sizes(oracle, monkeypatch, cid):
    """The measured order (candidate 3) with single-frame launches on two streams and alternating frame sizes,
    no rt_wait between them: rt_render_async frames on the library's async stream and rt_render_device frames on
    a torch stream, each size change recording the tile durations again and rebuilding the order while the other
    stream's launches may still read it (tile_order_prepare waits for the whole device first).  Every frame =
    the oracle's."""
    import torch
    monkeypatch.setenv("RT_DISPATCH_ORDER", "3")
    sizes = [(203, 117), (160, 96)]
    scs = [scenes.config(cid).resized(*s) for s in sizes]
    wants = [oracle.render(s, oracle.MODE_NEAREST, 8)[0] for s in scs]
    ctx = Context(1)
    hosts = [np.zeros(w * h, dtype=np.int32) for (w, h) in sizes for _ in range(3)]
    try:
        ctx.set_scene(scs[0])  # (the two sizes share the scene; rt_set_scene of either is the same tables)
        for hb in hosts:
            ctx.register_host(hb)
        W1, H1 = sizes[1]
        outs = [torch.zeros(W1 * H1, dtype=torch.int32, device="cuda") for _ in range(3)]
        s = torch.cuda.Stream()
        for k in range(3):
            ctx.render_async(*sizes[0], hosts[k])  # size 0, async stream
            ctx.render_device(W1, H1, outs[k].data_ptr(), s.cuda_stream)  # size 1, another stream
        ctx.wait()
        s.synchronize()
        for k in range(3):
            assert_same(hosts[k].reshape(sizes[0][1], sizes[0][0]), wants[0], f"{cid} async frame {k}")
            assert_same(outs[k].cpu().numpy().reshape(H1, W1), wants[1], f"{cid} device frame {k}")
        assert ctx.dispatch_order() == 3
    finally:
        for hb in hosts:
            ctx.unregister_host(hb)
        ctx.close()


@pytest.mark.parametrize("order", ["0", "3", None])
@pytest.mark.parametrize("cid", ["C2", "C3", "C4"])
def test_view_height_cut_frames_are_the_full_frames_rows(oracle, monkeypatch, cid, order):
    """rt_set_view_height (ABI 9): a W x H' render under a W x VH view (H' < VH) is rows [0, H') of the W x VH
    frame -- one-frame launches (rt_render, rt_render_device) under the dispatch orders 0 and 3 and the library's
    own choice, and band renders (8-row bands of 3 ranks into a row-major frame); H' > VH is an invalid argument.
    The direct kernel (C2, C3) and the bundle kernel (C4)."""
    import torch
    if order is None:
        monkeypatch.delenv("RT_DISPATCH_ORDER", raising=False)
    else:
        monkeypatch.setenv("RT_DISPATCH_ORDER", order)
    W, VH = 240, 136
    sc = scenes.config(cid).resized(W, VH)
    want, _ = oracle.render(sc, oracle.MODE_NEAREST, 8)
    ctx = Context(1)
    try:
        ctx.set_scene(sc)
        ctx.set_view_height(VH)
        st = torch.cuda.current_stream().cuda_stream
        for Hc in (VH, 99, 64, 1):
            for _ in range(2 if order is not None else 1):
                assert_same(ctx.render(W, Hc).copy(), want[:Hc], f"{cid} rt_render {W}x{Hc} of {W}x{VH}")
            out = torch.zeros(W * Hc, dtype=torch.int32, device="cuda")
            for k in range(60 if order is None else 2):  # (None: past the tuner's probes and its recording)
                ctx.render_device(W, Hc, out.data_ptr(), st)
                if k % 10 == 9:  # (the tuner reads its probes' events as they complete)
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            assert_same(out.cpu().numpy().reshape(Hc, W), want[:Hc], f"{cid} rt_render_device {W}x{Hc}")
            # the tuner's choice reads as made (the bundle kernel's cut frames are single-frame launches too; the
            # direct kernel's only at the full view height)
            if order is None and Hc > 8 and (cid == "C4" or Hc == VH):
                assert ctx.dispatch_order() in (0, 1, 2, 3), "a chosen order reads as still measuring"
            frame = torch.zeros(W * Hc, dtype=torch.int32, device="cuda")
            for r in range(3):
                ctx.render_bands_ex(W, Hc, 8, r, 3, frame.data_ptr(), abi.RT_BANDS_FRAME, st)
            torch.cuda.synchronize()
            assert_same(frame.cpu().numpy().reshape(Hc, W), want[:Hc], f"{cid} bands {W}x{Hc}")
        with pytest.raises(abi.RayTracerError) as ei:
            ctx.render(W, VH + 1)
        assert ei.value.code == abi.RT_ERR_INVALID_ARG
        ctx.set_view_height(0)  # back to the frame's own view
        small = scenes.config(cid).resized(W, 64)
        assert_same(ctx.render(W, 64).copy(), oracle.render(small, oracle.MODE_NEAREST, 8)[0], f"{cid} view reset")
    finally:
        ctx.close()


def test_reference_plugin_surface_tick_and_input(oracle):
    """RayTracer(Surface).Tick()/OnKeyPress/OnMouseMove, as template.cs drives it."""
    screen = Surface(128, 96)
    rt = RayTracer(screen)
    try:
        rt.Tick()
        want, _ = oracle.render(scenes.reference(128, 96), oracle.MODE_NEAREST, 4)
        assert_same(screen.image(), want, "Tick default camera")
        for key in ["W", "W", "A", "Space", "D", "LeftShift", "S", "Q"]:
            rt.OnKeyPress(key)
        rt.OnMouseMove(25.0, -12.0)
        rt.OnKeyPress("W")
        rt.Tick()
        sc = scenes.reference(128, 96)
        c = rt.camera
        sc.camera = (c.position.tuple(), c.yaw, c.pitch)
        want, _ = oracle.render(sc, oracle.MODE_NEAREST, 4)
        assert_same(screen.image(), want, "Tick moved camera")
    finally:
        rt.close()


def test_error_behaviour(rtlib):
    import ctypes as C
    ctx = Context(1)
    try:
        W = 16
        buf = np.zeros(W * W, dtype=np.int32)
        assert rtlib.rt_render(ctx.ptr, W, W, buf.ctypes.data) == abi.RT_ERR_NO_SCENE
        sc = scenes.reference(W, W)
        S, P, L = sc.c_arrays()
        rc = rtlib.rt_set_scene(ctx.ptr, S, 3, P, 1, L, 2, abi.rt_vec3(0, 0, 0), abi.RT_MAX_RECURSION_LIMIT + 1)
        assert rc == abi.RT_ERR_UNSUPPORTED and b"recursion_limit" in rtlib.rt_last_error(ctx.ptr)
        assert rtlib.rt_set_scene(ctx.ptr, S, -1, P, 1, L, 2, abi.rt_vec3(0, 0, 0), 1) == abi.RT_ERR_INVALID_ARG
        ctx.set_scene(sc)
        assert rtlib.rt_render(ctx.ptr, 0, W, buf.ctypes.data) == abi.RT_ERR_INVALID_ARG
        assert rtlib.rt_render(ctx.ptr, W, W, None) == abi.RT_ERR_INVALID_ARG
    finally:
        ctx.close()
    n = C.c_int(0)
    rtlib.rt_device_count(C.byref(n))
    p = C.c_void_p()
    assert rtlib.rt_create(n.value + 1, C.byref(p)) == abi.RT_ERR_NO_DEVICE


def test_stats_accumulate_and_reset(gpu_ctx, golden):
    e = golden["cases"]["C1"]
    sc = scenes.config("C1")
    gpu_ctx.set_scene(sc)
    gpu_ctx.reset_stats()
    for _ in range(3):
        gpu_ctx.render(sc.width, sc.height)
    st = gpu_ctx.stats()
    assert st["frames"] == 3 and st["launches"] == 3
    assert st["primary_rays"] == 3 * e["stats"]["primary_rays"]
    assert st["sphere_tests"] == (st["primary_rays"] + st["reflect_rays"] + st["shadow_rays"]) * 3
    assert st["kernel_ms"] > 0 and st["copy_ms"] > 0
    assert st["timed_launches"] == 1 and st["timed_copies"] == 1  # default: every 64th, first included
    gpu_ctx.reset_stats()
    assert gpu_ctx.stats()["primary_rays"] == 0


@pytest.mark.parametrize("cid", ["C2", "C4"])
def test_counting_off_same_pixels_no_rays(gpu_ctx, golden, cid):
    """rt_set_counting (ABI 10): with counting off a launch writes the same pixels (golden CRC, one-frame and
    4-frame batch launches, direct and bundle kernels) and adds frames / pixels / launches but no rays; on again,
    the counts resume exactly (the golden per-frame counts).  Only 0 and 1 are accepted."""
    e = golden["cases"][cid]
    sc = scenes.config(cid)
    W, H = sc.width, sc.height
    gpu_ctx.set_scene(sc)
    gpu_ctx.reset_stats()
    gpu_ctx.set_counting(False)
    try:
        assert crc(gpu_ctx.render(W, H)) == e["crc32"]
        import torch
        big = torch.empty(4 * W * H, dtype=torch.int32, device="cuda")
        st_ = torch.cuda.current_stream()
        gpu_ctx.render_bands_batch(W, H, 8, 0, 1, 4, big.data_ptr(), W * H * 4, abi.RT_BANDS_FRAME, st_.cuda_stream)
        torch.cuda.synchronize()
        frames = big.cpu().numpy().reshape(4, H, W)
        assert all(crc(f) == e["crc32"] for f in frames)
        st = gpu_ctx.stats()
        assert st["pixels"] == 5 * W * H and st["launches"] == 2
        assert st["primary_rays"] == st["reflect_rays"] == st["shadow_rays"] == 0 and st["sphere_tests"] == 0
    finally:
        gpu_ctx.set_counting(True)
    gpu_ctx.render(W, H)
    gpu_ctx.render_bands_batch(W, H, 8, 0, 1, 4, big.data_ptr(), W * H * 4, abi.RT_BANDS_FRAME, st_.cuda_stream)
    torch.cuda.synchronize()
    st = gpu_ctx.stats()
    want = {k: 5 * e["stats"][k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}
    assert ray_counts(st) == want and st["pixels"] == 10 * W * H
    for bad in (2, -1):
        assert gpu_ctx.lib.rt_set_counting(gpu_ctx.ptr, bad) == abi.RT_ERR_INVALID_ARG


def test_sampled_timing(gpu_ctx):
    sc = scenes.config("C1").resized(320, 180)
    gpu_ctx.set_scene(sc)
    for every, n, want in [(1, 5, 5), (2, 5, 3), (0, 5, 0), (64, 130, 3)]:
        gpu_ctx.set_timing(every)
        gpu_ctx.reset_stats()
        for _ in range(n):
            gpu_ctx.render(sc.width, sc.height)
        st = gpu_ctx.stats()
        assert st["launches"] == n and st["timed_launches"] == want and st["timed_copies"] == want
        assert (st["kernel_ms"] > 0) == (want > 0) and st["primary_rays"] == n * sc.width * sc.height
    with pytest.raises(Exception):
        gpu_ctx.set_timing(-1)
    gpu_ctx.set_timing(64)


def test_render_async_double_buffered_frames(oracle):
    """rt_render_async into two alternating host buffers with a new camera per frame
    (SURVEY 8f rank 1): every frame equals the oracle's frame for its own camera."""
    sc = scenes.reference(96, 72)
    W, H = sc.width, sc.height
    bufs = [np.zeros(W * H, dtype=np.int32) for _ in range(2)]
    cams = [((0.1 * k, 0.0, -0.2 * k), 0.07 * k, -0.03 * k) for k in range(6)]
    with Context(1) as ctx:
        ctx.set_scene(sc)
        for b in bufs:
            ctx.register_host(b)
        got = []
        for k, (pos, yaw, pitch) in enumerate(cams):
            ctx.set_camera(abi.rt_camera(abi.rt_vec3(*pos), yaw, pitch))
            ctx.render_async(W, H, bufs[k % 2])
            if k >= 1:  # frame k-1 is read after frame k is queued (rt_wait completes both: one in-order stream)
                ctx.wait()
                got.append(bufs[(k - 1) % 2].reshape(H, W).copy())
        ctx.wait()
        got.append(bufs[(len(cams) - 1) % 2].reshape(H, W).copy())
        for b in bufs:
            ctx.unregister_host(b)
    for k, (pos, yaw, pitch) in enumerate(cams):
        s2 = scenes.reference(W, H)
        s2.camera = (pos, float(np.float32(yaw)), float(np.float32(pitch)))
        want, _ = oracle.render(s2, oracle.MODE_NEAREST, 4)
        assert_same(got[k], want, f"async frame {k}")


def _oracle_frame(oracle, W, H, cam):
    pos, yaw, pitch = cam
    s2 = scenes.reference(W, H)
    s2.camera = (pos, float(np.float32(yaw)), float(np.float32(pitch)))
    return oracle.render(s2, oracle.MODE_NEAREST, 4)[0]


@pytest.mark.parametrize("inflight", [None, "0", "1", "3"])
def test_render_async_deep_queue_one_wait(oracle, monkeypatch, inflight):
    """rt_render_async under load -- 9 frames queued with a new camera each, each into
    its own registered host buffer, and one rt_wait at the end; the frame size changes twice
    mid-queue (reallocation of the device double buffer).  A missing or misplaced ordering between a
    frame's trace, its hand-off and the next trace into the same device buffer shows up as a wrong
    frame.  Under the default bound of 2 frames in flight (the call for frame k+2 waits for frame k's
    copy), without a bound, and at 1 and 3 (RT_TICK_INFLIGHT, read at rt_create)."""
    if inflight is None:
        monkeypatch.delenv("RT_TICK_INFLIGHT", raising=False)
    else:
        monkeypatch.setenv("RT_TICK_INFLIGHT", inflight)
    sizes = [(96, 72)] * 4 + [(130, 66)] * 3 + [(33, 17), (96, 72)]
    cams = [((0.1 * k, 0.05 * k, -0.2 * k), 0.07 * k, -0.03 * k) for k in range(len(sizes))]
    bufs = [np.full(w * h, 0x7f7f7f7f, dtype=np.int32) for w, h in sizes]
    with Context(1) as ctx:
        ctx.set_scene(scenes.reference(96, 72))
        for b in bufs:
            ctx.register_host(b)
        for (w, h), cam, b in zip(sizes, cams, bufs):
            ctx.set_camera(abi.rt_camera(abi.rt_vec3(*cam[0]), cam[1], cam[2]))
            ctx.render_async(w, h, b)
        ctx.wait()
        got = [b.reshape(h, w).copy() for (w, h), b in zip(sizes, bufs)]
        for b in bufs:
            ctx.unregister_host(b)
    for k, ((w, h), cam) in enumerate(zip(sizes, cams)):
        assert_same(got[k], _oracle_frame(oracle, w, h, cam), f"queued async frame {k} ({w}x{h})")


def test_render_async_full_hd_deep_queue(oracle):
    """The bench's Tick shape at 1920x1080: 5 queued frames, 2 alternating registered buffers
    would be overwritten, so 5 buffers; one wait; every frame = the oracle's for its camera."""
    W, H = 1920, 1080
    cams = [((0.0, 0.1 * k, -0.3 * k), 0.05 * k, 0.02 * k) for k in range(5)]
    bufs = [np.zeros(W * H, dtype=np.int32) for _ in cams]
    with Context(1) as ctx:
        ctx.set_scene(scenes.reference(W, H))
        for b in bufs:
            ctx.register_host(b)
        for cam, b in zip(cams, bufs):
            ctx.set_camera(abi.rt_camera(abi.rt_vec3(*cam[0]), cam[1], cam[2]))
            ctx.render_async(W, H, b)
        ctx.wait()
        got = [b.reshape(H, W).copy() for b in bufs]
        for b in bufs:
            ctx.unregister_host(b)
    for k, cam in enumerate(cams):
        assert_same(got[k], _oracle_frame(oracle, W, H, cam), f"1080p async frame {k}")


def test_render_async_unregistered_and_pinned_buffers(oracle):
    """Buffers not registered through rt_register_host (pageable numpy memory, torch's
    hipHostMalloc'd pinned memory) take hipMemcpyAsync on the same stream, never the copy slice:
    mixed in one queue with a registered buffer, every frame is right."""
    import torch
    W, H = 80, 60
    cams = [((0.0, 0.0, -0.1 * k), 0.1 * k, 0.0) for k in range(4)]
    reg = np.zeros(W * H, dtype=np.int32)
    pinned = torch.zeros(W * H, dtype=torch.int32, pin_memory=True)
    bufs = [np.zeros(W * H, dtype=np.int32), reg, pinned.numpy(), np.zeros(W * H, dtype=np.int32)]
    with Context(1) as ctx:
        ctx.set_scene(scenes.reference(W, H))
        ctx.register_host(reg)
        for cam, b in zip(cams, bufs):
            ctx.set_camera(abi.rt_camera(abi.rt_vec3(*cam[0]), cam[1], cam[2]))
            ctx.render_async(W, H, b)
        ctx.wait()
        got = [b.reshape(H, W).copy() for b in bufs]
        ctx.unregister_host(reg)
    for k, cam in enumerate(cams):
        assert_same(got[k], _oracle_frame(oracle, W, H, cam), f"async frame {k}")


def test_render_async_pending_frame_flushed_by_unregister_and_render(oracle):
    """A frame whose copy is still pending is written before rt_unregister_host releases its
    buffer and before a synchronous rt_render (which may reuse the buffer) runs."""
    W, H = 64, 48
    cam0, cam1 = ((0.2, 0.0, -0.5), 0.1, 0.05), ((-0.2, 0.1, -0.4), -0.1, 0.0)
    a = np.zeros(W * H, dtype=np.int32)
    b = np.zeros(W * H, dtype=np.int32)
    with Context(1) as ctx:
        ctx.set_scene(scenes.reference(W, H))
        ctx.register_host(a)
        ctx.register_host(b)
        ctx.set_camera(abi.rt_camera(abi.rt_vec3(*cam0[0]), cam0[1], cam0[2]))
        ctx.render_async(W, H, a)
        ctx.unregister_host(a)  # no rt_wait: the pending copy must land first
        got_a = a.reshape(H, W).copy()
        ctx.render_async(W, H, b)  # cam0 again, pending into b
        ctx.set_camera(abi.rt_camera(abi.rt_vec3(*cam1[0]), cam1[1], cam1[2]))
        ctx.render(W, H, b)  # the synchronous Tick into the same buffer: its frame must win
        got_b = b.reshape(H, W).copy()
        ctx.wait()
        assert np.array_equal(b.reshape(H, W), got_b), "a flushed async frame overwrote rt_render's"
        ctx.unregister_host(b)
    assert_same(got_a, _oracle_frame(oracle, W, H, cam0), "frame pending at rt_unregister_host")
    assert_same(got_b, _oracle_frame(oracle, W, H, cam1), "rt_render after a pending async frame")


@pytest.mark.parametrize("cid,w,h", [("REF", 96, 64), ("C3", 80, 45), ("C4", 64, 36)])
def test_debug_segments_match_visible_path_ray_counts(gpu_ctx, oracle, cid, w, h):
    """rt_debug_segments with stride 1: one segment per visible-path ray,
    so the per-kind counts equal the oracle's primary / reflect / shadow ray counts."""
    sc = scenes.config(cid).resized(w, h)
    gpu_ctx.set_scene(sc)
    segs, total = gpu_ctx.debug_segments(w, h, sample_stride=1, capacity=w * h * 64)
    _, st = oracle.render(sc, oracle.MODE_NEAREST, 4)
    assert total == len(segs)
    kinds = np.bincount(segs["kind"], minlength=3)
    assert kinds.tolist() == [st["primary_rays"], st["reflect_rays"], st["shadow_rays"]]
    assert (segs["pixel"] >= 0).all() and (segs["pixel"] < w * h).all()
    prim = segs[segs["kind"] == 0]
    assert np.array_equal(np.sort(prim["pixel"]), np.arange(w * h))
    cam = np.array(sc.camera[0], dtype=np.float32)
    assert (prim["ox"] == cam[0]).all() and (prim["oy"] == cam[1]).all() and (prim["oz"] == cam[2]).all()
    for f in ("ox", "oy", "oz", "ex", "ey", "ez"):
        assert np.isfinite(segs[f]).all()


def test_debug_segments_stride_and_capacity(gpu_ctx):
    sc = scenes.reference(100, 60)
    gpu_ctx.set_scene(sc)
    segs, total = gpu_ctx.debug_segments(100, 60, sample_stride=7, capacity=100 * 60)
    prim = segs[segs["kind"] == 0]
    assert len(prim) == -(-6000 // 7) and (prim["pixel"] % 7 == 0).all()
    small, total2 = gpu_ctx.debug_segments(100, 60, sample_stride=7, capacity=10)
    assert total2 == total and len(small) == 10  # a full buffer keeps the count of every append
    import ctypes as C
    n = C.c_int(0)
    lib = gpu_ctx.lib
    assert lib.rt_debug_segments(gpu_ctx.ptr, 100, 60, 0, None, 0, C.byref(n)) == abi.RT_ERR_INVALID_ARG
    assert lib.rt_debug_segments(gpu_ctx.ptr, 100, 60, 1, None, 5, C.byref(n)) == abi.RT_ERR_INVALID_ARG
    assert lib.rt_debug_segments(gpu_ctx.ptr, 100, 60, 1, None, 0, C.byref(n)) == abi.RT_OK and n.value > 6000


def test_debug_tick_composites_inset_over_exact_frame(oracle):
    """RayTracer(debug=True).Tick(): the DEBUG_ENABLE frame -- outside the inset every pixel
    is the traced pixel or a white circle point; inside only inset colours."""
    from raytracer_hip import DebugView, debugview
    screen = Surface(160, 120)
    rt = RayTracer(screen, debug=True)
    try:
        rt.Tick()
    finally:
        rt.close()
    want, _ = oracle.render(scenes.reference(160, 120), oracle.MODE_NEAREST, 4)
    img = screen.image()
    v = DebugView(160, 120)
    inset = v.inset_mask()  # black: x > TopLeftX && y > TopLeftY
    lines = np.zeros_like(inset)  # ClampToDebugView is inclusive of TopLeft
    lines[v.top_left_y:, v.top_left_x:] = True
    diff = ~lines & (img != want)
    assert (img[diff] == debugview.CIRCLE_COLOR).all()
    edge = lines & ~inset & (img != want)
    assert set(np.unique(img[edge]).tolist()) <= {debugview.CIRCLE_COLOR, *debugview.KIND_COLORS.values()}
    colours = set(np.unique(img[inset]).tolist())
    assert colours <= {0, debugview.CIRCLE_COLOR, *debugview.KIND_COLORS.values()}
    assert colours & set(debugview.KIND_COLORS.values())


def test_set_scene_waits_for_frames_in_flight(gpu_ctx, golden):
    """rt_set_scene right after rt_render_device on a caller stream (no host sync): the
    in-flight frame must still see the old scene (the upload waits for the device)."""
    import torch
    a, b = golden["cases"]["C3_96x54"], golden["cases"]["C1_64"]
    sa, sb = scenes.config(a["config"]).resized(a["width"], a["height"]), scenes.config(b["config"]).resized(
        b["width"], b["height"])
    outs = []
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for k in range(6):
            sc = sa if k % 2 == 0 else sb
            gpu_ctx.set_scene(sc)
            out = torch.empty(sc.width * sc.height, dtype=torch.int32, device="cuda")
            gpu_ctx.render_device(sc.width, sc.height, out.data_ptr(), s.cuda_stream)
            outs.append(out)
    s.synchronize()
    for k, out in enumerate(outs):
        e = a if k % 2 == 0 else b
        assert crc(out.cpu().numpy()) == e["crc32"], k


def test_two_frames_in_flight_on_two_streams(gpu_ctx, golden):
    """bench.py's swap chain: frames alternate between two streams and buffers."""
    import torch
    e = golden["cases"]["C2_96x54"]
    sc = scenes.config(e["config"]).resized(e["width"], e["height"])
    gpu_ctx.set_scene(sc)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.full((sc.width * sc.height,), -1, dtype=torch.int32, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    for k in range(10):
        gpu_ctx.render_device(sc.width, sc.height, outs[k % 2].data_ptr(), streams[k % 2].cuda_stream)
    torch.cuda.synchronize()
    assert all(crc(o.cpu().numpy()) == e["crc32"] for o in outs)


def _segment_scenes():
    from random_scenes import camera_sweep_scene, random_scene
    out = [scenes.reference(96, 64), scenes.config("C3").resized(80, 45), scenes.config("C4").resized(64, 36)]
    out += [random_scene(s) for s in range(8)] + [random_scene(s, dense=True) for s in range(100, 104)]
    out += [camera_sweep_scene(s, 96, 64) for s in range(0, 12)]
    return out


@pytest.mark.parametrize("k", list(range(27)))
def test_debug_segments_are_the_oracle_hit_records(gpu_ctx, oracle, k):
    """Float hit records, 0 ulp: every visible-path segment of every pixel --
    origin, hit point / shadow-blocker point, kind -- bit-identical to oracle_segments."""
    sc = _segment_scenes()[k]
    want = oracle.segments(sc)
    gpu_ctx.set_scene(sc)
    got, total = gpu_ctx.debug_segments(sc.width, sc.height, sample_stride=1, capacity=len(want) + 64)
    assert total == len(want)
    got = got[np.argsort(got["pixel"], kind="stable")]  # per-lane appends keep each pixel's order
    if got.tobytes() != want.tobytes():
        diff = np.nonzero([a.tobytes() != b.tobytes() for a, b in zip(got, want)])[0]
        i = int(diff[0])
        pytest.fail(f"{sc.name}: {len(diff)} of {len(want)} records differ; first #{i}: gpu {got[i]} oracle {want[i]}")


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("fmt", [0, 1])
def test_band_sets_and_one_launch_reassembly(gpu_ctx, golden, world, fmt):
    """rt_render_bands_ex (int32 / RGB24) per simulated rank into one gathered buffer, then
    rt_scatter_gathered: the full frame, bit-exact."""
    import torch
    e = golden["cases"]["C3_96x54"]
    sc = scenes.config(e["config"]).resized(e["width"], e["height"])
    W, H, br = sc.width, sc.height, 8
    gpu_ctx.set_scene(sc)
    bpp = 4 if fmt == 0 else 3
    stride = (bands_of(H, br, 0, world) * br * W * bpp + 255) // 256 * 256 + 512  # padded like dist.py
    g = torch.full((world * stride,), 0xEE, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for r in range(world):
        gpu_ctx.render_bands_ex(W, H, br, r, world, g.data_ptr() + r * stride, fmt, s)
    frame = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
    gpu_ctx.scatter_gathered(W, H, br, world, g.data_ptr(), stride, frame.data_ptr(), fmt, s)
    torch.cuda.synchronize()
    assert crc(frame.cpu().numpy()) == e["crc32"]
