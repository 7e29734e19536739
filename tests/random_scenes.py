"""Seeded random scenes for GPU-vs-oracle parity (tests only).

They deliberately exercise every branch of RayTracer.cs: all five material factories plus
arbitrary material mixes, generic specular exponents (the f64 Math.Pow path), planes with
arbitrary normals (including +-x normals, where the checkerboard basis is NaN, Q11), lights
at the origin (a shadow ray with a zero direction), cameras inside spheres and moved/rotated
cameras.
"""
from __future__ import annotations

import numpy as np

from raytracer_hip import scenes
from raytracer_hip.scenes import Light, Material, Plane, Scene, Sphere

f32 = np.float32


def _v(rng, lo, hi):
    return tuple(float(f32(x)) for x in rng.uniform(lo, hi, 3))


def _color(rng):
    return tuple(float(f32(x)) for x in rng.integers(0, 256, 3) / 255.0)


def _material(rng):
    k = rng.integers(0, 7)
    c = _color(rng)
    if k == 0:
        return Material.diffuse(c)
    if k == 1:
        return Material.plastic(c, float(f32(rng.choice([1.0, 0.5, 2.0, 3.7, 12.0]))))
    if k == 2:
        return Material.metal(c, float(f32(rng.choice([0.5, 1.0, 7.25]))))
    if k == 3:
        return Material.mirror(_color(rng) if rng.random() < 0.5 else scenes.ONE)
    if k == 4:
        return Material.diffuse_mirror(c, _v(rng, 0.1, 0.9))
    if k == 5:  # everything at once
        return Material(c, _color(rng), _color(rng), float(f32(rng.uniform(0.1, 20))), _v(rng, 0.0, 0.6))
    return Material((0.0, 0.0, 0.0), _color(rng), (0.0, 0.0, 0.0), 0.0, (0.0, 0.0, 0.0))  # ambient only


def random_scene(seed: int, width: int = 96, height: int = 64, dense: bool = False) -> Scene:
    """dense=True: 12-100 smaller spheres -- exercises the wave-bundle culling path
    (CULL_MIN_SPHERES = 12) and its 64-sphere chunking."""
    rng = np.random.default_rng(seed)
    ns = int(rng.integers(12, 101)) if dense else int(rng.integers(0, 12))
    spheres = []
    for _ in range(ns):
        r = float(f32(rng.uniform(0.05, 0.9) if dense else rng.uniform(0.2, 2.0)))
        spheres.append(Sphere(_v(rng, -6, 6)[:2] + (float(f32(rng.uniform(1, 24))),), r, _material(rng)))
    planes = []
    for _ in range(int(rng.integers(0, 3))):
        kind = rng.integers(0, 4)
        if kind == 0:
            n = (0.0, 1.0, 0.0)
        elif kind == 1:
            n = (1.0, 0.0, 0.0) if rng.random() < 0.5 else (-1.0, 0.0, 0.0)  # NaN checkerboard basis
        else:
            v = rng.normal(size=3)
            v = v / np.linalg.norm(v)
            n = tuple(float(f32(x)) for x in v)
        planes.append(Plane(_v(rng, -3, 3), n, _material(rng)))
    lights = []
    for _ in range(int(rng.integers(0, 4))):
        pos = (0.0, 0.0, 0.0) if rng.random() < 0.15 else _v(rng, -30, 30)
        lights.append(Light(pos, float(f32(rng.uniform(0.2, 1.5)))))
    limit = int(rng.choice([0, 1, 2, 3, 5, 9, 32]))
    amb = (float(f32(rng.uniform(0, 0.3))),) * 3
    cam_pos = _v(rng, -1, 1)
    if spheres and rng.random() < 0.1:
        cam_pos = spheres[0].center  # camera inside a sphere
    cam = (cam_pos, float(f32(rng.uniform(-0.6, 0.6))), float(f32(rng.uniform(-0.4, 0.4))))
    return Scene(f"rand{seed}", width, height, spheres, planes, lights, amb, limit, cam)


def camera_sweep_scene(seed: int, width: int = 160, height: int = 96) -> Scene:
    """Views for the per-frame primary screen boxes (view_params): spheres all around the
    camera, any yaw/pitch, cameras far from the origin, inside or touching spheres, huge and
    tiny spheres, extreme aspect ratios -- every silhouette must match the oracle."""
    rng = np.random.default_rng(10_000 + seed)
    mode = seed % 5
    cam_pos = _v(rng, -2, 2)
    if mode == 1:  # far from the origin (direction error of vp - cam grows with |cam|)
        cam_pos = tuple(float(f32(c * 10.0 ** rng.integers(2, 5))) for c in _v(rng, -1, 1))
    ns = int(rng.integers(1, 64))
    spheres = []
    for k in range(ns):
        off = rng.normal(size=3)
        off *= rng.uniform(0.5, 30) / np.linalg.norm(off)
        r = float(f32(10.0 ** rng.uniform(-2.5, 0.8)))
        c = tuple(float(f32(cam_pos[j] + off[j])) for j in range(3))
        if mode == 2 and k == 0:  # camera inside the first sphere
            c, r = cam_pos, 3.0
        if mode == 3 and k == 0:  # camera on the first sphere's surface
            c = (float(f32(cam_pos[0] + 1.0)), cam_pos[1], cam_pos[2])
            r = 1.0
        spheres.append(Sphere(c, r, _material(rng)))
    lights = [Light(_v(rng, -30, 30), float(f32(rng.uniform(0.2, 1.5)))) for _ in range(int(rng.integers(0, 3)))]
    planes = []
    if seed % 2 == 0:  # mirror planes: first reflections use the per-frame mirror boxes
        for _ in range(int(rng.integers(1, 4))):
            v = rng.normal(size=3)
            v = v / np.linalg.norm(v)
            n = tuple(float(f32(x)) for x in v)
            off = rng.normal(size=3)
            off *= rng.uniform(0.5, 12) / np.linalg.norm(off)
            c = tuple(float(f32(cam_pos[j] + off[j])) for j in range(3))
            km = _v(rng, 0.3, 1.0)
            mat = Material.mirror(km) if rng.random() < 0.5 else Material.diffuse_mirror(_color(rng), km)
            planes.append(Plane(c, n, mat))
    if mode == 4:
        width, height = (int(rng.integers(1, 9)), int(rng.integers(40, 200))) if rng.random() < 0.5 else \
            (int(rng.integers(40, 300)), int(rng.integers(1, 9)))
    yaw = float(f32(rng.uniform(-7, 7)))
    pitch = float(f32(rng.uniform(-1.6, 1.6)))
    limit = int(rng.choice([0, 1, 3]))
    return Scene(f"sweep{seed}", width, height, spheres, planes, lights, (0.1, 0.1, 0.1), limit, (cam_pos, yaw, pitch))
