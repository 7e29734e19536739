"""Independent float32 emulation of Raytracer/RayTracer.cs (tests only).

Written directly from the C# source, separately from oracle/oracle.c, to cross-check
the C restatement: vectorised over pixels with numpy float32 arrays (every elementwise
op is one correctly-rounded binary32 operation, as SSE scalar code), double precision
where the C# goes through Math.* (libm via Python's math module), and the reference's
full ALL-HIT structure: every primitive is traced and shaded, recursing into
TraceSecondaryRay for every mirror hit, exactly as RayTracer.cs:729-1002 does.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32
f64 = np.float64
INT_MIN = np.int32(-2147483648)
ZERO = f32(0.0)


class V3:
    """OpenTK.Mathematics.Vector3 over arrays (or scalars) of float32."""
    __slots__ = ("x", "y", "z")

    def __init__(self, x, y, z):
        self.x, self.y, self.z = f32(x) if np.isscalar(x) else x, f32(y) if np.isscalar(y) else y, \
            f32(z) if np.isscalar(z) else z

    def __add__(self, o):
        return V3(self.x + o.x, self.y + o.y, self.z + o.z)

    def __sub__(self, o):
        return V3(self.x - o.x, self.y - o.y, self.z - o.z)

    def mul(self, o):  # Vector3 * Vector3 (componentwise)
        return V3(self.x * o.x, self.y * o.y, self.z * o.z)

    def scale(self, s):  # Vector3 * float
        return V3(self.x * s, self.y * s, self.z * s)

    def take(self, idx):
        g = lambda a: a[idx] if not np.isscalar(a) and np.ndim(a) else a
        return V3(g(self.x), g(self.y), g(self.z))

    def bcast(self, n):
        b = lambda a: np.full(n, a, dtype=f32) if np.ndim(a) == 0 else a
        return V3(b(self.x), b(self.y), b(self.z))


def dot(a, b):
    return (a.x * b.x + a.y * b.y) + a.z * b.z


def length(a):
    return np.sqrt((a.x * a.x + a.y * a.y) + a.z * a.z)


def normalize(a):
    with np.errstate(all="ignore"):
        s = f32(1.0) / length(a)
        return V3(a.x * s, a.y * s, a.z * s)


def cross(l, r):
    return V3(l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x)


def net_max(a, b):
    """System.Math.Max(float, float): IEEE 754-2019 maximum."""
    a = np.asarray(a, dtype=f32)
    b = np.asarray(b, dtype=f32)
    ne = np.where(np.isnan(a), a, np.where(b < a, a, b))
    eq = np.where(np.signbit(b), a, b)
    return np.where(a != b, ne, eq).astype(f32)


def net_min(a, b):
    a = np.asarray(a, dtype=f32)
    b = np.asarray(b, dtype=f32)
    ne = np.where(np.isnan(a), a, np.where(a < b, a, b))
    eq = np.where(np.signbit(a), a, b)
    return np.where(a != b, ne, eq).astype(f32)


def net_to_int(v):
    """(int)x on .NET 6 x64: truncation, NaN / out of range -> int.MinValue."""
    v = np.asarray(v, dtype=f64)
    ok = (v > -2147483649.0) & (v < 2147483648.0)
    return np.where(ok, np.trunc(np.where(ok, v, 0.0)), -2147483648.0).astype(np.int64).astype(np.int32)


def is_zero(c):
    return c[0] == 0 and c[1] == 0 and c[2] == 0


class Mat:
    def __init__(self, m):
        self.kd, self.ka, self.ks = (V3(*m.kd), V3(*m.ka), V3(*m.ks))
        self.n = f32(m.n)
        self.km = V3(*m.km)
        self.is_mirror = not is_zero(m.km)            # :85
        self.is_diffuse = not is_zero(m.kd)           # :89
        self.has_spec = (not is_zero(m.ks)) and self.n > 0  # :93


class Emu:
    def __init__(self, scene):
        self.sc = scene
        self.spheres = [(V3(*s.center), f32(s.radius) * f32(s.radius), Mat(s.material)) for s in scene.spheres]
        self.planes = [(V3(*p.center), V3(*p.normal), Mat(p.material)) for p in scene.planes]
        self.lights = [(V3(*l.position), f32(l.intensity)) for l in scene.lights]
        self.ambient = V3(*scene.ambient)
        self.limit = scene.recursion_limit

    # IntersectsSphere, :613-642
    def isect_sphere(self, o, d, center, r2, eps=ZERO):
        oc = o - center
        a = dot(d, d)
        b = f32(2) * dot(oc, d)
        c = dot(oc, oc) - r2
        disc = b * b - (f32(4) * a) * c
        hit = disc >= 0
        with np.errstate(all="ignore"):
            ds = np.sqrt(disc.astype(f64)).astype(f32)
            a2 = f32(2) * a
            d2 = (-b + ds) / a2
            d1 = (-b - ds) / a2
        dist = net_min(net_max(d1, ZERO), net_max(d2, ZERO))
        dist_eps = net_min(net_max(d1 - eps, ZERO), net_max(d2 - eps, ZERO))
        col = hit & (dist_eps > 0)
        return col, np.where(col, dist, ZERO).astype(f32)

    # IntersectPlane, :590-604
    def isect_plane(self, o, d, center, normal):
        with np.errstate(all="ignore"):
            t = (((-o.x) * normal.x - o.y * normal.y) - o.z * normal.z + dot(center, normal)) / dot(d, normal)
        col = t > 0
        return col, np.where(col, t, ZERO).astype(f32)

    # IntersectShadowLight, :573-582
    def shadow(self, hp, light):
        pos, inten = light
        blocked = np.zeros(hp.x.shape, dtype=bool)
        for (c, r2, _m) in self.spheres:
            col, _ = self.isect_sphere(hp, pos, c, r2, f32(0.001))
            blocked |= col
        return np.where(blocked, ZERO, inten).astype(f32)

    # ShapePhongShading, :665-695
    def phong(self, hp, ray_d, normal, m, light):
        pos, _ = light
        L = normalize(pos - hp)
        Vw = normalize(ray_d)
        n = hp.x.shape[0]
        diff = V3(ZERO, ZERO, ZERO).bcast(n)
        if m.is_diffuse:
            ang = dot(normal, L)
            diff = m.kd.scale(net_max(ZERO, ang)).bcast(n)
        spec = V3(ZERO, ZERO, ZERO).bcast(n)
        if m.has_spec:
            Rs = L - normal.scale(f32(2) * dot(L, normal))
            sp = dot(Vw, normalize(Rs))
            base = net_max(ZERO, sp).astype(f64)
            pw = np.array([math.pow(float(x), float(m.n)) if not math.isnan(x) else math.nan for x in base],
                          dtype=f64).astype(f32)
            spec = m.ks.mul(V3(pw, pw, pw))
        return diff + spec

    @staticmethod
    def reflect(v, nrm):  # CalculateReflectionRay, :718-720
        return v - nrm.scale(f32(2) * dot(v, nrm))

    # TracePlane, :729-780
    def trace_plane(self, o, d, plane, count):
        center, normal, m = plane
        n = o.x.shape[0]
        col, dist = self.isect_plane(o, d, center, normal)
        color = V3(np.zeros(n, f32), np.zeros(n, f32), np.zeros(n, f32))
        shade = col & ~(dist - f32(0.01) <= 0)
        if count > self.limit:
            one = np.where(shade, f32(1), ZERO).astype(f32)
            return dist, V3(one, one.copy(), one.copy())
        idx = np.nonzero(shade)[0]
        if idx.size == 0:
            return dist, color
        o_, d_, t_ = o.take(idx), d.take(idx), dist[idx]
        hp = o_ + d_.scale(t_)
        c = V3(np.zeros(idx.size, f32), np.zeros(idx.size, f32), np.zeros(idx.size, f32))
        if m.is_mirror:
            sec = self.trace_secondary(hp, self.reflect(d_, normal.bcast(idx.size)), count + 1)
            c = c + sec.mul(m.km)
        if m.is_diffuse:
            for light in self.lights:
                li = self.shadow(hp, light)
                att = np.array([1.0 / math.pow(float(t), 2) for t in t_], dtype=f64).astype(f32)
                e1 = normalize(cross(normal, V3(1, 0, 0)))
                if e1.x == 0 and e1.y == 0 and e1.z == 0:
                    e1 = normalize(cross(normal, V3(0, 0, 1)))
                e2 = normalize(cross(normal, e1))
                u = dot(e1.bcast(idx.size), hp)
                v = dot(e2.bcast(idx.size), hp)
                chk = ((net_to_int(u).astype(np.int64) + net_to_int(v).astype(np.int64)) & 1).astype(f32)
                term = V3(li, li, li).scale(att).mul(self.phong(hp, d_, normal.bcast(idx.size), m, light)).mul(
                    V3(chk, chk, chk))
                c = c + V3(net_max(term.x, ZERO), net_max(term.y, ZERO), net_max(term.z, ZERO))
        c = c + self.ambient.mul(m.ka).bcast(idx.size)
        for comp in ("x", "y", "z"):
            getattr(color, comp)[idx] = getattr(c, comp)
        return dist, color

    # TraceSphere, :835-876
    def trace_sphere(self, o, d, sphere, count):
        center, r2, m = sphere
        n = o.x.shape[0]
        col, dist = self.isect_sphere(o, d, center, r2)
        color = V3(np.zeros(n, f32), np.zeros(n, f32), np.zeros(n, f32))
        shade = col & ~(dist - f32(0.01) <= 0)
        if count > self.limit:
            return dist, color
        idx = np.nonzero(shade)[0]
        if idx.size == 0:
            return dist, color
        o_, d_, t_ = o.take(idx), d.take(idx), dist[idx]
        hp = o_ + d_.scale(t_)
        c = V3(np.zeros(idx.size, f32), np.zeros(idx.size, f32), np.zeros(idx.size, f32))
        if m.is_mirror:
            nrm = normalize(hp - center.bcast(idx.size))
            c = c + self.trace_secondary(hp, self.reflect(d_, nrm), count + 1).mul(m.km)
        if m.is_diffuse:
            for light in self.lights:
                li = self.shadow(hp, light)
                att = f32(1) / t_ * t_
                nrm = normalize(hp - center.bcast(idx.size))
                c = c + V3(li, li, li).scale(att).mul(self.phong(hp, d_, nrm, m, light))
        c = c + self.ambient.mul(m.ka).bcast(idx.size)
        for comp in ("x", "y", "z"):
            getattr(color, comp)[idx] = getattr(c, comp)
        return dist, color

    # TraceSecondaryRay, :789-826
    def trace_secondary(self, hp, d, count):
        n = hp.x.shape[0]
        best_s = np.full(n, np.inf, f32)
        sc = V3(np.zeros(n, f32), np.zeros(n, f32), np.zeros(n, f32))
        for sp in self.spheres:
            dist, col = self.trace_sphere(hp, d, sp, count)
            sel = (dist - f32(0.01) > 0) & (dist - f32(0.01) < best_s)
            best_s = np.where(sel, dist, best_s)
            sc = V3(np.where(sel, col.x, sc.x), np.where(sel, col.y, sc.y), np.where(sel, col.z, sc.z))
        best_p = np.full(n, np.inf, f32)
        pc = V3(np.zeros(n, f32), np.zeros(n, f32), np.zeros(n, f32))
        for pl in self.planes:
            dist, col = self.trace_plane(hp, d, pl, count)
            sel = (dist > 0) & (dist < best_p)
            best_p = np.where(sel, dist, best_p)
            pc = V3(np.where(sel, col.x, pc.x), np.where(sel, col.y, pc.y), np.where(sel, col.z, pc.z))
        pick = best_s < best_p
        return V3(np.where(pick, sc.x, pc.x), np.where(pick, sc.y, pc.y), np.where(pick, sc.z, pc.z))

    # Camera, :511-523 and Tick :892-896
    def camera(self):
        (pos, yaw, pitch) = self.sc.camera
        p, y = float(f32(pitch)), float(f32(yaw))
        F = V3(f32(math.cos(p) * math.sin(y)), f32(-math.sin(p)), f32(math.cos(p) * math.cos(y)))
        R = V3(f32(math.cos(y)), f32(0), f32(-math.sin(y)))
        U = cross(R, F)
        deg2rad = f32(math.pi) / f32(180)
        rad = f32(60) * f32(0.5) * deg2rad
        ph = f32(0.3) * f32(math.tan(float(rad))) * f32(2)
        aspect = f32(self.sc.width) / f32(self.sc.height)
        pw = ph * aspect
        return V3(*pos), R, U, F, V3(pw, ph, f32(0.3))

    # TracePixel, :962-1002, for every pixel of rows [r0, r1)
    def render(self, rows=None):
        W, H = self.sc.width, self.sc.height
        r0, r1 = rows or (0, H)
        cam, R, U, F, vp = self.camera()
        ys, xs = np.mgrid[r0:r1, 0:W]
        xs, ys = xs.ravel(), ys.ravel()
        px = xs.astype(f32) / f32(W) - f32(0.5)
        py = ys.astype(f32) / f32(H) - f32(0.5)
        n = xs.size
        local = V3(px, py, np.full(n, f32(1))).mul(vp)
        point = ((cam.bcast(n) + R.scale(local.x)) + U.scale(local.y)) + F.scale(local.z)
        d = normalize(point - cam.bcast(n))
        o = cam.bcast(n)
        best_s = np.full(n, np.inf, f32)
        sc = V3(np.zeros(n, f32), np.zeros(n, f32), np.zeros(n, f32))
        for sp in self.spheres:
            dist, col = self.trace_sphere(o, d, sp, 0)
            sel = (dist > 0) & (best_s > dist)
            best_s = np.where(sel, dist, best_s)
            sc = V3(np.where(sel, col.x, sc.x), np.where(sel, col.y, sc.y), np.where(sel, col.z, sc.z))
        best_p = np.full(n, np.inf, f32)
        pc = V3(np.zeros(n, f32), np.zeros(n, f32), np.zeros(n, f32))
        for pl in self.planes:
            dist, col = self.trace_plane(o, d, pl, 0)
            sel = (dist > 0) & (best_p > dist)
            best_p = np.where(sel, dist, best_p)
            pc = V3(np.where(sel, col.x, pc.x), np.where(sel, col.y, pc.y), np.where(sel, col.z, pc.z))
        pick = best_s < best_p
        col = V3(np.where(pick, sc.x, pc.x), np.where(pick, sc.y, pc.y), np.where(pick, sc.z, pc.z))
        return shift_color(col).reshape(r1 - r0, W)


def shift_color(c):
    """ShiftColor, :1046-1052: Math.Clamp (NaN passes), *255f, Math.Floor (double), (int), (byte)."""
    def chan(v):
        v = np.asarray(v, dtype=f32)
        cl = np.where(v < 0, ZERO, np.where(v > 1, f32(1), v)).astype(f32)
        fl = np.floor((cl * f32(255)).astype(f64))
        return (net_to_int(fl).astype(np.int64) & 0xFF)
    r, g, b = chan(c.x), chan(c.y), chan(c.z)
    return ((r << 16) | (g << 8) | b).astype(np.int32)
