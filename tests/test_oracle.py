"""CPU oracle: known-answer tests derived by hand from Raytracer/RayTracer.cs, its two
drivers against each other, the independent numpy float32 emulation, and the committed
golden fixtures.  (No GPU; the reference ships no tests of its own -- parity unpinned.)"""
import math
import os
import zlib

import numpy as np
import pytest

from raytracer_hip import abi, scenes

V = abi.rt_vec3
INT_MIN = -2147483648


def test_intersect_sphere_kat(oracle):
    l = oracle.lib()
    col = __import__("ctypes").c_int(0)
    # ray down +z from the origin through a unit sphere at z=5: roots 4 and 6 -> 4 (:613-642)
    t = l.oracle_intersect_sphere(V(0, 0, 0), V(0, 0, 1), V(0, 0, 5), 1.0, 0.0, col)
    assert col.value == 1 and t == 4.0
    # origin inside the sphere: one root negative -> distance 0 -> miss (Q7)
    t = l.oracle_intersect_sphere(V(0, 0, 5), V(0, 0, 1), V(0, 0, 5), 1.0, 0.0, col)
    assert col.value == 0 and t == 0.0
    # shadow ray starting on the surface: t1 = 0 -> 0 - 0.001 < 0 -> not an obstruction
    t = l.oracle_intersect_sphere(V(0, 0, 4), V(0, 0, 1), V(0, 0, 5), 1.0, 0.001, col)
    assert col.value == 0
    # sphere behind the ray: both roots negative -> miss
    t = l.oracle_intersect_sphere(V(0, 0, 0), V(0, 0, -1), V(0, 0, 5), 1.0, 0.0, col)
    assert col.value == 0 and t == 0.0
    # unnormalised direction (shadow rays use the light POSITION as direction, :574)
    t = l.oracle_intersect_sphere(V(0, 0, 0), V(0, 0, 2), V(0, 0, 5), 1.0, 0.001, col)
    assert col.value == 1 and t == 2.0


def test_intersect_plane_kat(oracle):
    l = oracle.lib()
    col = __import__("ctypes").c_int(0)
    t = l.oracle_intersect_plane(V(0, 0, 0), V(0, -1, 0), V(0, -1, 0), V(0, 1, 0), col)
    assert col.value == 1 and t == 1.0
    # parallel ray: numerator -1, denominator +0 -> -inf -> miss (the 512^2 centre pixel)
    t = l.oracle_intersect_plane(V(0, 0, 0), V(0, 0, 1), V(0, -1, 0), V(0, 1, 0), col)
    assert col.value == 0 and t == 0.0
    # plane above the origin looking down its normal: t > 0 only in front
    t = l.oracle_intersect_plane(V(0, 0, 0), V(0, 1, 0), V(0, -1, 0), V(0, 1, 0), col)
    assert col.value == 0


def test_shift_color_kat(oracle):
    l = oracle.lib()
    # NaN -> (int)NaN = int.MinValue -> (byte) 0; 2 -> clamp 1 -> 255; -1 -> 0 (:1046-1052)
    assert l.oracle_shift_color(V(float("nan"), 2.0, -1.0)) == 0x0000FF00
    assert l.oracle_shift_color(V(1.0, 0.5, 0.0)) == 0x00FF7F00
    assert l.oracle_shift_color(V(-0.0, 0.999, 1e-9)) == 0x0000FE00


def test_net_float_to_int(oracle):
    l = oracle.lib()
    assert l.oracle_net_float_to_int(float("nan")) == INT_MIN
    assert l.oracle_net_float_to_int(3e9) == INT_MIN
    assert l.oracle_net_float_to_int(-3e9) == INT_MIN
    assert l.oracle_net_float_to_int(-2.75) == -2
    assert l.oracle_net_float_to_int(2147483520.0) == 2147483520
    assert l.oracle_net_float_to_int(-2147483648.0) == INT_MIN


def test_camera_default_basis(oracle):
    """Default camera: F=(0,-0,1), R=(1,0,-0), U=(0,-1,-0) -> image row 0 looks up (:511-523)."""
    l = oracle.lib()
    v = abi.rt_view()
    cam = abi.rt_camera(V(0, 0, 0), 0.0, 0.0)
    assert l.oracle_camera_view(cam, 512, 512, v) == 0
    assert v.forward.tuple() == (0.0, 0.0, 1.0) and math.copysign(1, v.forward.y) < 0
    assert v.right.tuple() == (1.0, 0.0, 0.0) and math.copysign(1, v.right.z) < 0
    assert v.up.tuple() == (0.0, -1.0, 0.0)
    ph = np.float32(0.3) * np.float32(math.tan(float(np.float32(30.0) * (np.float32(math.pi) / np.float32(180)))))
    assert v.plane_height == float(ph * np.float32(2))
    assert v.near_clip == float(np.float32(0.3))


def test_centre_pixel_black(oracle):
    """512^2 centre pixel: ray (0,+0,~1) misses all spheres and the plane (t = -1/+0)."""
    sc = scenes.reference(512, 512)
    px, _ = oracle.render(sc, oracle.MODE_REFERENCE, 1, rows=(256, 257))
    assert px[0, 256] == 0


@pytest.mark.parametrize("cfg,w,h", [("REF", 48, 48), ("C1", 48, 32), ("C2", 80, 45), ("C3", 80, 45),
                                     ("C4", 48, 27)])
def test_oracle_vs_numpy_emulation(oracle, cfg, w, h):
    import emu_f32
    sc = scenes.config(cfg).resized(w, h)
    ref, _ = oracle.render(sc, oracle.MODE_REFERENCE, 4)
    near, _ = oracle.render(sc, oracle.MODE_NEAREST, 4)
    emu = emu_f32.Emu(sc).render()
    assert np.array_equal(ref, near)
    assert np.array_equal(ref, emu), f"{int((ref != emu).sum())} pixels differ from the float32 emulation"


def test_oracle_vs_emulation_moved_camera(oracle):
    import emu_f32
    sc = scenes.reference(64, 48)
    sc.camera = ((0.35, 0.2, -0.4), 0.3, -0.15)
    ref, _ = oracle.render(sc, oracle.MODE_REFERENCE, 4)
    near, _ = oracle.render(sc, oracle.MODE_NEAREST, 4)
    emu = emu_f32.Emu(sc).render()
    assert np.array_equal(ref, near) and np.array_equal(ref, emu)


def test_oracle_golden_raw_frames(oracle, golden):
    import os
    for cid, e in golden["cases"].items():
        if "frame" not in e:
            continue
        sc = scenes.config(e["config"]).resized(e["width"], e["height"])
        px, st = oracle.render(sc, oracle.MODE_NEAREST)
        want = np.load(os.path.join(os.path.dirname(__file__), "golden", e["frame"]))
        assert np.array_equal(px, want), cid
        assert st == e["stats"], cid


@pytest.mark.parametrize("cid", ["REF_512", "REF_1280x720", "C1", "C2", "C3"])
def test_oracle_golden_crc(oracle, golden, cid):
    e = golden["cases"][cid]
    sc = scenes.config(e["config"]).resized(e["width"], e["height"])
    px, st = oracle.render(sc, oracle.MODE_NEAREST)
    assert f"{zlib.crc32(px.tobytes()) & 0xFFFFFFFF:08x}" == e["crc32"]
    assert st == e["stats"]


def test_oracle_rows_subset(oracle):
    sc = scenes.config("C1").resized(64, 64)
    full, _ = oracle.render(sc, oracle.MODE_NEAREST, 2)
    part, _ = oracle.render(sc, oracle.MODE_REFERENCE, 3, rows=(10, 37))
    assert np.array_equal(full[10:37], part)


@pytest.mark.parametrize("seed", list(range(0, 40, 3)))
def test_random_scenes_oracle_vs_emulation(oracle, seed):
    """Seeded random scenes (every material kind, generic Math.Pow exponents, +-x plane normals,
    lights at the origin, cameras inside spheres): both oracle drivers == numpy emulation."""
    import emu_f32
    import random_scenes
    sc = random_scenes.random_scene(seed, 48, 32)
    ref, _ = oracle.render(sc, oracle.MODE_REFERENCE, 4)
    near, _ = oracle.render(sc, oracle.MODE_NEAREST, 4)
    with np.errstate(all="ignore"):
        emu = emu_f32.Emu(sc).render()
    assert np.array_equal(ref, near) and np.array_equal(ref, emu)


@pytest.mark.parametrize("seed", [100, 107, 115])
def test_dense_random_scenes_oracle_drivers(oracle, seed):
    """Dense scenes (the GPU culling path's inputs): all-hit and nearest-hit drivers agree."""
    import random_scenes
    sc = random_scenes.random_scene(seed, 64, 48, dense=True)
    ref, _ = oracle.render(sc, oracle.MODE_REFERENCE, 4)
    near, _ = oracle.render(sc, oracle.MODE_NEAREST, 4)
    assert np.array_equal(ref, near)


@pytest.mark.parametrize("cid,w,h", [("REF", 96, 64), ("C3", 80, 45), ("C4", 48, 27)])
def test_oracle_segments_count_every_visible_ray(oracle, cid, w, h):
    """oracle_segments (float hit records): one record per visible-path ray."""
    from raytracer_hip import scenes
    sc = scenes.config(cid).resized(w, h)
    seg = oracle.segments(sc)
    _, st = oracle.render(sc, oracle.MODE_NEAREST, 2)
    assert np.bincount(seg["kind"], minlength=3).tolist() == [st["primary_rays"], st["reflect_rays"],
                                                                 st["shadow_rays"]]
    prim = seg[seg["kind"] == 0]
    assert np.array_equal(prim["pixel"], np.arange(w * h))
    assert np.all(np.diff(seg["pixel"]) >= 0)  # walk order, pixel by pixel


def test_full_size_goldens_pinned_by_the_all_hit_driver():
    """tests/golden/pin_allhit.log (make_golden.py --pin): every full-size golden CRC -- C4 3840x2160 and
    C5 7680x4320 included -- was re-derived by the reference-faithful all-hit driver (every hit shaded,
    RayTracer.cs:975-991, 792-823) and equals the nearest driver's and golden.json's, and the numpy
    emulation agrees on the C4/C5 scene at 384x216.  The log must cover every golden full-size case."""
    import json
    import re
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    gold = json.load(open(os.path.join(here, "golden.json")))["cases"]
    log = open(os.path.join(here, "pin_allhit.log")).read().splitlines()
    seen = {}
    for line in log:
        m = re.match(r"(\S+)\s+(\d+)x(\d+) all-hit ([0-9a-f]{8}) nearest ([0-9a-f]{8}) golden ([0-9a-f]{8}) "
                     r"mismatching pixels (\d+) (OK|FAIL)", line)
        if m:
            seen[m.group(1)] = m
    for cid in ("REF_512", "REF_1280x720", "C1", "C2", "C3", "C4", "C5"):
        m = seen[cid]
        assert m.group(8) == "OK" and m.group(7) == "0"
        assert m.group(4) == m.group(5) == m.group(6) == gold[cid]["crc32"], cid
        assert (int(m.group(2)), int(m.group(3))) == (gold[cid]["width"], gold[cid]["height"])
    assert any(line.startswith("C4/C5 scene") and line.rstrip().split()[-3] == "OK" for line in log)
