#!/usr/bin/env python3
"""CPU model (float64, statistics only -- never a parity reference) of the bundle kernel's shadow
culling on a BASELINE config: traces sampled 8x8 tiles through the nearest-hit walk, and for every
(tile, fold level) with diffuse records compares the candidate sets of

  ball  -- the in-tree cull: one ShadowSphere bound per level (make_shadow_sphere) and per light
           shadow_sphere_cull's line / behind rules with their margins (rt_kernel.hip);
  grid  -- per-lane lookups: a per-light 2-D grid of 64-bit candidate masks over the light frame's
           (u, v) plane, ANDed with a per-light axial table (spheres whose centre lies ahead of the
           lane's axial coordinate), OR-reduced over the wave.

Reports per wave and level: candidates per light, the union over lights, and the (sphere, light)
pairs the merged pass would visit (upper bound, no early exit).  Usage:
  python tools/shadow_cull_model.py [--config C4] [--stride 3] [--grid 64,128,256] [--slabs 64]
"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))
from raytracer_hip import scenes  # noqa: E402


def light_frame(p):
    """rt_api.cpp rt_set_scene: the shadow-cull frame (U, V, A) of a light position."""
    p = np.asarray(p, dtype=np.float64)
    n = np.linalg.norm(p)
    A = p / n if n > 0 else np.array([0.0, 0.0, 1.0])
    h = np.array([1.0, 0.0, 0.0]) if abs(A[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
    U = np.cross(A, h)
    U /= np.linalg.norm(U)
    V = np.cross(A, U)
    return U, V, A


def trace(sc, xs, ys):
    """Nearest-hit walk of pixels (xs, ys): per level the hit point, 'diffuse record' flag, active."""
    W, H = sc.width, sc.height
    near, fov = 0.3, 60.0
    ph = near * math.tan(math.radians(fov / 2)) * 2
    pw = ph * (W / H)
    lx = (xs / W - 0.5) * pw
    ly = (ys / H - 0.5) * ph
    # yaw = pitch = 0: right (1,0,0), up (0,-1,0), forward (0,0,1)
    d = np.stack([lx, -ly, np.full_like(lx, near)], axis=1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.zeros_like(d)
    C = np.array([s.center for s in sc.spheres])
    r2 = np.array([s.radius ** 2 for s in sc.spheres])
    smat = [s.material for s in sc.spheres]
    s_mirror = np.array([any(m.km) for m in smat])
    s_diff = np.array([any(m.kd) for m in smat])
    PC = np.array([p.center for p in sc.planes])
    PN = np.array([p.normal for p in sc.planes])
    p_mirror = np.array([any(p.material.km) for p in sc.planes])
    p_diff = np.array([any(p.material.kd) for p in sc.planes])
    n = len(xs)
    active = np.ones(n, bool)
    levels = []
    for count in range(sc.recursion_limit + 2):
        oc = o[:, None, :] - C[None]
        b = 2 * np.einsum("nsk,nk->ns", oc, d)
        c = np.einsum("nsk,nsk->ns", oc, oc) - r2[None]
        disc = b * b - 4 * c
        with np.errstate(invalid="ignore"):
            t1 = (-b - np.sqrt(np.where(disc >= 0, disc, np.nan))) / 2
        ok = (t1 > 0) if count == 0 else (t1 - 0.01 > 0)
        t1 = np.where(ok, t1, np.inf)
        si = np.argmin(t1, axis=1)
        ts = t1[np.arange(n), si]
        den = d @ PN.T
        with np.errstate(divide="ignore", invalid="ignore"):
            tp = (np.einsum("pk,pk->p", PC, PN)[None] - o @ PN.T) / den
        tp = np.where(tp > 0, tp, np.inf)
        pi = np.argmin(tp, axis=1)
        tpl = tp[np.arange(n), pi]
        is_s = ts < tpl
        t = np.where(is_s, ts, tpl)
        hit = active & np.isfinite(t) & (t - 0.01 > 0)
        if count > sc.recursion_limit:
            break
        hp = o + d * t[:, None]
        mirror = np.where(is_s, s_mirror[si], p_mirror[pi]) & hit
        diff = np.where(is_s, s_diff[si], p_diff[pi]) & hit
        levels.append((hp, diff, hit))
        nrm = np.where(is_s[:, None], hp - C[si], PN[pi])
        nrm = np.where(is_s[:, None], nrm / np.linalg.norm(nrm, axis=1, keepdims=True), nrm)
        d = d - nrm * (2 * np.einsum("nk,nk->n", d, nrm))[:, None]
        o = hp
        active = mirror
        if not active.any():
            break
    return levels


def ball_masks(hp, C, rr_c, frames):
    """In-tree cull of one wave level: hp (k, 3) diffuse hit points -> [mask per light] (bool (S,))."""
    a, b = hp[0], hp[-1]
    O = (a + b) / 2
    R = np.linalg.norm(hp - O, axis=1).max() * (1 + 2 ** -10) + 2 ** -60
    omgn = 2 ** -18 * np.linalg.norm(O) * (1 + 2 ** -10)
    out = []
    for (U, V, A), shc in frames:
        ou, ov, oa = O @ U, O @ V, O @ A
        wu, wv, wa = shc[:, 0] - ou, shc[:, 1] - ov, shc[:, 2] - oa
        dc = np.abs(wu) + np.abs(wv) + np.abs(wa)
        mgn = 2 ** -8 * (dc + 3 * R) + omgn
        T = R + shc[:, 3] + mgn
        line = wu * wu + wv * wv > T * T
        behind = -wa - R > mgn
        out.append(~(line | behind))
    return out


class Grid:
    """Per-light (u, v) grid of candidate masks + axial 'ahead' table, for lanes with |hp|_1 <= B."""

    def __init__(self, frame, shc, G, slabs, B):
        U, V, A = frame
        self.frame = frame
        cu, cv, ca, rr = shc[:, :4].T
        clen1 = np.abs(shc[:, 4])  # |C|_1
        # margin for any lane with |hp|_1 <= B: 2^-8 (|C - hp|_1) + 2^-18 |hp| <= 2^-8 (|C|_1 + B) + 2^-18 B
        self.T = rr + 2 ** -8 * (clen1 + B) + 2 ** -18 * B
        self.B = B
        lo_u, hi_u = (cu - self.T).min(), (cu + self.T).max()
        lo_v, hi_v = (cv - self.T).min(), (cv + self.T).max()
        self.u0, self.v0 = lo_u, lo_v
        self.cs_u, self.cs_v = (hi_u - lo_u) / G, (hi_v - lo_v) / G
        self.G = G
        # cell (i, j) rect; sphere in cell iff distance(centre, rect) <= T
        gu = lo_u + np.arange(G + 1) * self.cs_u
        gv = lo_v + np.arange(G + 1) * self.cs_v
        du = np.maximum(0, np.maximum(gu[:-1, None] - cu[None], cu[None] - gu[1:, None]))  # (G, S)
        dv = np.maximum(0, np.maximum(gv[:-1, None] - cv[None], cv[None] - gv[1:, None]))
        self.cell = (du[:, None, :] ** 2 + dv[None, :, :] ** 2) <= self.T[None, None, :] ** 2  # (G, G, S)
        # axial: a sphere can block only if b < 0, i.e. its centre lies ahead: ca - a_hp > -margin
        self.ca = ca + 2 ** -8 * (clen1 + B) + 2 ** -18 * B
        self.slabs = slabs
        self.a0, self.a1 = self.ca.min(), self.ca.max()
        self.cs_a = (self.a1 - self.a0) / slabs if slabs else 1.0
        edges = self.a0 + np.arange(slabs) * self.cs_a  # slab k covers [a0 + k cs, a0 + (k+1) cs)
        self.slab = self.ca[None, :] > edges[:, None] if slabs else None  # (slabs, S)
        self.ca_raw = ca
        self.cmax1 = clen1.max()
        self.bu0, self.bu1 = (cu - rr).min(), (cu + rr).max()
        self.bv0, self.bv1 = (cv - rr).min(), (cv + rr).max()

    def masks(self, hp):
        """Per-lane candidate masks of hit points hp (k, 3) -> (wave OR, any lane on the fallback).
        A lane whose (u, v) lies outside the bounding box of every sphere's disc -- grown by its own
        margin 2^-8 (|hp|_1 + max |C|_1) -- has no candidate; a lane beyond the table's bound
        (|hp|_1 > B) inside that box takes every sphere ahead of it."""
        U, V, A = self.frame
        u, v, a = hp @ U, hp @ V, hp @ A
        l1 = np.abs(hp).sum(axis=1)
        far = l1 > self.B
        iu = np.floor((u - self.u0) / self.cs_u).astype(np.int64)
        iv = np.floor((v - self.v0) / self.cs_v).astype(np.int64)
        m = self.cell[np.clip(iu, 0, self.G - 1), np.clip(iv, 0, self.G - 1)]
        outside = (iu < 0) | (iu >= self.G) | (iv < 0) | (iv >= self.G)
        m = np.where(outside[:, None], False, m)
        if self.slabs:
            ia = np.floor((a - self.a0) / self.cs_a).astype(np.int64)
            ahead = np.where((ia < 0)[:, None], True, self.slab[np.clip(ia, 0, self.slabs - 1)])
            ahead = np.where((ia >= self.slabs)[:, None], False, ahead)
        else:
            ahead = np.ones_like(m)
        # far lanes: own margin, bbox test only
        mg = 2 ** -8 * (l1 + self.cmax1) + 2 ** -18 * l1
        inbox = ((u > self.bu0 - mg) & (u < self.bu1 + mg) & (v > self.bv0 - mg) & (v < self.bv1 + mg))
        fall = far & inbox
        m = np.where(far[:, None], fall[:, None], m & ahead)  # far lane in the box: every sphere
        return m.any(axis=0), fall.any()


def ahead_far(g, a, l1):
    """Far lanes: spheres whose centre lies ahead, with the lane's own margin (every sphere when unknown)."""
    mg = 2 ** -8 * (l1 + g.cmax1) + 2 ** -18 * l1
    return g.ca_raw[None, :] + mg[:, None] > a[:, None]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--stride", type=int, default=3, help="every n-th tile in x and y")
    ap.add_argument("--grid", default="32,64,128")
    ap.add_argument("--slabs", default="0,64")
    ap.add_argument("--bound", type=float, default=64.0)
    ap.add_argument("--bounds", default="", help="comma list of lane bounds B (overrides --bound)")
    args = ap.parse_args()
    sc = scenes.config(args.config)
    W, H = sc.width, sc.height
    C = np.array([s.center for s in sc.spheres], dtype=np.float64)
    rr_c = np.array([np.nextafter(np.float32(math.sqrt(np.float32(s.radius) ** 2) * (1 + 2 ** -8)), np.float32(np.inf))
                     for s in sc.spheres], dtype=np.float64)
    frames = []
    for l in sc.lights:
        U, V, A = light_frame(l.position)
        clen = np.linalg.norm(C, axis=1)
        shc = np.stack([C @ U, C @ V, C @ A, rr_c + 2 ** -18 * clen, np.abs(C).sum(axis=1)], axis=1)
        frames.append(((U, V, A), shc))
    tiles_x, tiles_y = (W + 7) // 8, (H + 7) // 8
    tx = np.arange(0, tiles_x, args.stride)
    ty = np.arange(0, tiles_y, args.stride)
    lane = np.arange(64)
    TX, TY = np.meshgrid(tx, ty, indexing="ij")
    TX, TY = TX.ravel(), TY.ravel()
    bounds = [float(b) for b in args.bounds.split(",")] if args.bounds else [args.bound]
    grids = {(G, s, int(B)): [Grid(f, shc, G, s, B) for f, shc in frames]
             for G in map(int, args.grid.split(",")) for s in map(int, args.slabs.split(",")) if G > 0
             for B in bounds}
    L = len(sc.lights)
    stats = {"ball": np.zeros((8, 3)), "lane": np.zeros((8, 3)), "split2": np.zeros((8, 3)),
             **{k: np.zeros((8, 3)) for k in grids}}
    lanes_lv = np.zeros(8)
    waves_lv = np.zeros(8)
    far_lv = {k: np.zeros(8) for k in grids}
    chunk = 1024
    for c0 in range(0, len(TX), chunk):
        ctx_, cty = TX[c0:c0 + chunk], TY[c0:c0 + chunk]
        xs = (ctx_[:, None] * 8 + (lane & 7)[None]).ravel().astype(np.float64)
        ys = (cty[:, None] * 8 + (lane >> 3)[None]).ravel().astype(np.float64)
        levels = trace(sc, xs, ys)
        for li_, (hp, diff, _) in enumerate(levels):
            hp = hp.reshape(-1, 64, 3)
            diff = diff.reshape(-1, 64)
            for w in range(hp.shape[0]):
                dm = diff[w]
                if not dm.any():
                    continue
                h = hp[w][dm]
                waves_lv[li_] += 1
                lanes_lv[li_] += len(h)
                lane_m = [np.logical_or.reduce(z) for z in zip(*[ball_masks(h[i:i + 1], C, rr_c, frames)
                                                                 for i in range(len(h))])]
                half = max(1, len(h) // 2)
                parts = [h[:half], h[half:]] if len(h) > 1 else [h]
                split_m = [np.logical_or.reduce(z) for z in zip(*[ball_masks(q, C, rr_c, frames) for q in parts])]
                for key, masks in [("ball", ball_masks(h, C, rr_c, frames)), ("lane", lane_m),
                                   ("split2", split_m)] + [
                        (k, [g.masks(h)[0] for g in gs]) for k, gs in grids.items()]:
                    per = sum(int(m.sum()) for m in masks)
                    uni = int(np.logical_or.reduce(masks).sum())
                    stats[key][li_] += (per / L, uni, per)
                for k, gs in grids.items():
                    far_lv[k][li_] += any(g.masks(h)[1] for g in gs)
    print(f"# {sc.name} {W}x{H}, tiles every {args.stride}: {len(TX)} waves sampled; per wave-level with diffuse "
          f"records: mean candidates per light / union / (sphere, light) pairs; grid = (cells per side, axial slabs); "
          f"lane bound |hp|_1 <= {args.bound}")
    nl = int((waves_lv > 0).sum())
    print("diffuse lanes per wave-level:", " ".join(f"{lanes_lv[i] / max(1, waves_lv[i]):.1f}" for i in range(8)
                                                     if waves_lv[i]))
    print("levels with diffuse records per sampled wave:", " ".join(f"{waves_lv[i] / len(TX):.3f}" for i in range(nl)))
    for key, s in stats.items():
        tot = s[:nl].sum(axis=0) / len(TX)
        row = " ".join(f"L{i}:{s[i, 0] / max(1, waves_lv[i]):5.2f}/{s[i, 1] / max(1, waves_lv[i]):5.2f}"
                       f"/{s[i, 2] / max(1, waves_lv[i]):5.2f}" for i in range(nl))
        extra = ""
        if key in far_lv:
            extra = f"  fallback-levels/wave {far_lv[key][:nl].sum() / len(TX):.3f}"
        print(f"{str(key):>10}: per wave pairs {tot[2]:6.2f} union {tot[1]:6.2f} | {row}{extra}")


if __name__ == "__main__":
    main()
