"""Scene presets: the reference scene (RayTracer.cs:441-469) and the synthetic
benchmark configurations of BASELINE.json / SURVEY.md 8(d), from a seeded,
deterministic generator.

Every value is built in float32 exactly as the reference's constructors would build it
(e.g. the ambient colour is 43f/255f, RayTracer.cs:469; colour bytes are b/255f).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import abi

F = np.float32


def f32(x) -> float:
    return float(F(x))


def vec(x, y, z) -> tuple:
    return (f32(x), f32(y), f32(z))


ZERO = (0.0, 0.0, 0.0)
ONE = (1.0, 1.0, 1.0)


@dataclass(frozen=True)
class Material:
    """RayTracer.cs:60-110; factories :117-158."""
    kd: tuple
    ka: tuple
    ks: tuple
    n: float
    km: tuple

    @staticmethod
    def diffuse(c):
        return Material(c, c, ZERO, 0.0, ZERO)

    @staticmethod
    def plastic(c, n=1.0):
        return Material(c, c, vec(0.4, 0.4, 0.4), f32(n), ZERO)

    @staticmethod
    def metal(c, n=1.0):
        return Material(c, c, c, f32(n), ZERO)

    @staticmethod
    def mirror(km):
        return Material(ZERO, ZERO, ZERO, 0.0, km)

    @staticmethod
    def diffuse_mirror(c, km):
        return Material(c, c, ZERO, 0.0, km)


@dataclass(frozen=True)
class Sphere:
    center: tuple
    radius: float
    material: Material


@dataclass(frozen=True)
class Plane:
    center: tuple
    normal: tuple
    material: Material


@dataclass(frozen=True)
class Light:
    position: tuple
    intensity: float


@dataclass
class Scene:
    name: str
    width: int
    height: int
    spheres: list
    planes: list
    lights: list
    ambient: tuple
    recursion_limit: int
    camera: tuple = (ZERO, 0.0, 0.0)  # (position, yaw, pitch): RayTracer.cs:494-502 defaults
    note: str = ""
    meta: dict = field(default_factory=dict)

    def resized(self, width: int, height: int, name: str | None = None) -> "Scene":
        return Scene(name or f"{self.name}@{width}x{height}", width, height, list(self.spheres),
                     list(self.planes), list(self.lights), self.ambient, self.recursion_limit,
                     self.camera, self.note, dict(self.meta))

    # ---- ctypes marshalling -------------------------------------------------
    def c_arrays(self):
        def m(mt: Material):
            return abi.rt_material(abi.rt_vec3(*mt.kd), abi.rt_vec3(*mt.ka), abi.rt_vec3(*mt.ks),
                                   mt.n, abi.rt_vec3(*mt.km))

        S = (abi.rt_sphere * max(1, len(self.spheres)))(
            *[abi.rt_sphere(abi.rt_vec3(*s.center), s.radius, m(s.material)) for s in self.spheres])
        P = (abi.rt_plane * max(1, len(self.planes)))(
            *[abi.rt_plane(abi.rt_vec3(*p.center), abi.rt_vec3(*p.normal), m(p.material)) for p in self.planes])
        L = (abi.rt_light * max(1, len(self.lights)))(
            *[abi.rt_light(abi.rt_vec3(*l.position), l.intensity) for l in self.lights])
        return S, P, L

    def c_camera(self):
        pos, yaw, pitch = self.camera
        return abi.rt_camera(abi.rt_vec3(*pos), f32(yaw), f32(pitch))


# ---- the reference scene, RayTracer.cs:441-469 --------------------------------
REF_SPHERES = [
    Sphere(vec(2.5, 0, 8), 1.0, Material.diffuse(vec(1, 0, 0))),
    Sphere(vec(3, 0, 5), 1.0, Material.plastic(vec(0, 1, 0))),
    Sphere(vec(-3, 1, 8), 1.0, Material.mirror(vec(1, 1, 1))),
]
REF_LIGHTS = [Light(vec(-3, 1, -3), 1.0), Light(vec(33, 1, 10), 1.0)]
REF_PLANES = [
    Plane(vec(0, -1, 0), vec(0, 1, 0),
          Material(vec(1, 1, 1), vec(0.5, 0.5, 0.5), ONE, f32(0.5), vec(1, 1, 1))),
]
REF_AMBIENT = (f32(F(43) / F(255)),) * 3
REF_LIMIT = 32  # ReflectionRecursionLimit, RayTracer.cs:490


# ---- seeded generator -------------------------------------------
class SplitMix64:
    MASK = (1 << 64) - 1

    def __init__(self, seed: int):
        self.state = seed & self.MASK

    def next(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & self.MASK
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.MASK
        return z ^ (z >> 31)

    def uniform(self) -> float:
        return (self.next() >> 40) * 2.0 ** -24


def _q(x: float) -> float:
    """Quantise to 1/64 (exactly representable in float32)."""
    return math.floor(64.0 * x + 0.5) / 64.0


def generated_spheres(count: int, seed: int = 0x5EED) -> list:
    """Spheres 3..count-1 after the three reference spheres."""
    rng = SplitMix64(seed)
    out = list(REF_SPHERES[:min(3, count)])
    for i in range(3, count):
        r = _q(0.25 + 0.75 * rng.uniform())
        x = _q(-8.0 + 16.0 * rng.uniform())
        z = _q(4.0 + 28.0 * rng.uniform())
        y = _q(-1.0 + r + 0.5 * rng.uniform())
        col = tuple(f32(F(rng.next() >> 56) / F(255)) for _ in range(3))
        kind = i % 5
        if kind == 0:
            mt = Material.diffuse(col)
        elif kind == 1:
            mt = Material.plastic(col, 1.0)
        elif kind == 2:
            mt = Material.metal(col, 0.5)
        elif kind == 3:
            mt = Material.mirror(ONE)
        else:
            mt = Material.diffuse_mirror(col, vec(0.5, 0.5, 0.5))
        out.append(Sphere(vec(x, y, z), f32(r), mt))
    return out


C4_LIGHTS = [Light(vec(-3, 1, -3), 1.0), Light(vec(33, 1, 10), 1.0), Light(vec(0, 12, 4), 1.0),
             Light(vec(-20, 6, 30), f32(0.8))]
C4_PLANES = REF_PLANES + [Plane(vec(0, 0, 48), vec(0, 0, -1), Material.diffuse(vec(0.6, 0.6, 0.6)))]


def reference(width=512, height=512) -> Scene:
    """The verbatim reference scene: 3 spheres, 1 plane, 2 lights, limit 32."""
    return Scene("ref", width, height, list(REF_SPHERES), list(REF_PLANES), list(REF_LIGHTS),
                 REF_AMBIENT, REF_LIMIT, note="RayTracer.cs:441-490 verbatim")


def config(name: str) -> Scene:
    """BASELINE.json configs.  depth D <=> recursion limit D-1."""
    name = name.upper()
    if name == "REF":
        return reference()
    if name == "REF720":
        return reference(1280, 720).resized(1280, 720, "REF720")  # the reference window, template.cs:65
    if name == "C1":
        return Scene("C1", 512, 512, list(REF_SPHERES), list(REF_PLANES), REF_LIGHTS[:1], REF_AMBIENT, 0,
                     note="512x512, 3 spheres + 1 plane, 1 light, depth 1")
    if name == "C2":
        return Scene("C2", 1920, 1080, generated_spheres(8), list(REF_PLANES), REF_LIGHTS[:1], REF_AMBIENT, 0,
                     note="1920x1080, 8 spheres + 1 plane, 1 light, depth 1")
    if name == "C3":
        return Scene("C3", 1920, 1080, generated_spheres(8), list(REF_PLANES), list(REF_LIGHTS), REF_AMBIENT, 3,
                     note="1920x1080, 8 spheres + 1 plane, 2 lights, depth 4")
    if name == "C4":
        return Scene("C4", 3840, 2160, generated_spheres(64), list(C4_PLANES), list(C4_LIGHTS), REF_AMBIENT, 5,
                     note="3840x2160, 64 spheres + 2 planes, 4 lights, depth 6")
    if name == "C5":
        return Scene("C5", 7680, 4320, generated_spheres(64), list(C4_PLANES), list(C4_LIGHTS), REF_AMBIENT, 5,
                     note="7680x4320, C4 scene, depth 6 (multi-GPU row tiles)")
    raise KeyError(name)


CONFIGS = ["C1", "C2", "C3", "C4", "C5"]
