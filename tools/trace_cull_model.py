#!/usr/bin/env python3
"""CPU model (float64, statistics only) of the bundle kernel's reflected-segment culling: per wave
(8x8 tile) and reflected segment, the candidate spheres of the wave bundle (make_bundle +
cull_mask: origin ball R, direction cone delta, line / behind rules with their margins) against
the spheres that some lane's ray actually reaches (disc >= 0 and b < 0: no cull can drop them).
    python tools/trace_cull_model.py [--config C4] [--stride 12]"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))
from raytracer_hip import scenes  # noqa: E402


def walk(sc, xs, ys):
    """Per reflected segment k >= 1: (o, d, active) of every pixel (nearest-hit walk)."""
    W, H = sc.width, sc.height
    near = 0.3
    ph = near * math.tan(math.radians(30)) * 2
    pw = ph * (W / H)
    d = np.stack([(xs / W - 0.5) * pw, -(ys / H - 0.5) * ph, np.full(len(xs), near)], axis=1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.zeros_like(d)
    C = np.array([s.center for s in sc.spheres])
    r2 = np.array([s.radius ** 2 for s in sc.spheres])
    s_mirror = np.array([any(s.material.km) for s in sc.spheres])
    PC = np.array([p.center for p in sc.planes])
    PN = np.array([p.normal for p in sc.planes])
    p_mirror = np.array([any(p.material.km) for p in sc.planes])
    n = len(xs)
    active = np.ones(n, bool)
    segs = []
    prev = np.full(n, -1)
    for count in range(sc.recursion_limit + 1):
        if count > 0:
            segs.append((o.copy(), d.copy(), active.copy(), prev.copy()))
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
        with np.errstate(divide="ignore", invalid="ignore"):
            tp = (np.einsum("pk,pk->p", PC, PN)[None] - o @ PN.T) / (d @ PN.T)
        tp = np.where(tp > 0, tp, np.inf)
        pi = np.argmin(tp, axis=1)
        tpl = tp[np.arange(n), pi]
        is_s = ts < tpl
        t = np.where(is_s, ts, tpl)
        hit = active & np.isfinite(t) & (t - 0.01 > 0)
        hp = o + d * np.where(np.isfinite(t), t, 0)[:, None]
        mirror = np.where(is_s, s_mirror[si], p_mirror[pi]) & hit
        nrm = np.where(is_s[:, None], hp - C[si], PN[pi])
        nrm = np.where(is_s[:, None], nrm / np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30), nrm)
        d = d - nrm * (2 * np.einsum("nk,nk->n", d, nrm))[:, None]
        o = hp
        prev = np.where(is_s, si, -1 - pi)
        active = mirror
        if not active.any():
            break
    return segs


def bundle_cull(o, d, C, rr):
    """make_bundle + cull_mask (rt_kernel.hip) for the active lanes' rays (k, 3) -> candidate mask (S,)."""
    O = (o[0] + o[-1]) / 2
    A = d[0] / np.linalg.norm(d[0])
    R = np.linalg.norm(o - O, axis=1).max() * (1 + 2 ** -10) + 2 ** -60
    dn = d / np.linalg.norm(d, axis=1, keepdims=True)
    delta = np.linalg.norm(dn - A, axis=1).max() * (1 + 2 ** -10) + 2 ** -20
    if delta >= 0.5:
        return np.ones(len(C), bool)
    w = C - O
    dc = np.linalg.norm(w, axis=1) * (1 + 2 ** -20)
    mgn = 2 ** -8 * (dc + R)
    x = np.linalg.norm(np.cross(w, A), axis=1)
    line = (x - dc * delta - R) > rr + mgn
    behind = (-(w @ A) - dc * delta - R * (1 + delta)) > mgn
    return ~(line | behind)


def reachable(o, d, C, r2):
    """Spheres some lane's ray reaches (disc >= 0, b < 0)."""
    oc = o[:, None, :] - C[None]
    b = 2 * np.einsum("ksj,kj->ks", oc, d)
    c = np.einsum("ksj,ksj->ks", oc, oc) - r2[None]
    a = np.einsum("kj,kj->k", d, d)[:, None]
    return ((b * b - 4 * a * c >= 0) & (b < 0)).any(axis=0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--stride", type=int, default=12)
    a = ap.parse_args()
    sc = scenes.config(a.config)
    C = np.array([s.center for s in sc.spheres])
    r2 = np.array([s.radius ** 2 for s in sc.spheres])
    rr = np.sqrt(r2) * (1 + 2 ** -8)
    tx = np.arange(0, (sc.width + 7) // 8, a.stride)
    ty = np.arange(0, (sc.height + 7) // 8, a.stride)
    TX, TY = [v.ravel() for v in np.meshgrid(tx, ty, indexing="ij")]
    lane = np.arange(64)
    L = sc.recursion_limit
    cnt = np.zeros((L + 1, 6))  # waves, active lanes, bundle candidates, reachable, split by previous primitive, groups
    for c0 in range(0, len(TX), 1024):
        xs = (TX[c0:c0 + 1024, None] * 8 + (lane & 7)[None]).ravel().astype(float)
        ys = (TY[c0:c0 + 1024, None] * 8 + (lane >> 3)[None]).ravel().astype(float)
        for k, (o, d, act, pv) in enumerate(walk(sc, xs, ys), start=1):
            o, d, act, pv = o.reshape(-1, 64, 3), d.reshape(-1, 64, 3), act.reshape(-1, 64), pv.reshape(-1, 64)
            for w in range(o.shape[0]):
                m = act[w]
                if not m.any():
                    continue
                # split: the lanes that reflected off the first active lane's primitive, then the rest
                first = pv[w][m][0]
                g1 = m & (pv[w] == first)
                g2 = m & ~g1
                split = bundle_cull(o[w][g1], d[w][g1], C, rr).sum() + (
                    bundle_cull(o[w][g2], d[w][g2], C, rr).sum() if g2.any() else 0)
                cnt[k] += (1, m.sum(), bundle_cull(o[w][m], d[w][m], C, rr).sum(), reachable(o[w][m], d[w][m], C, r2).sum(),
                           split, 1 + g2.any())
    print(f"# {sc.name}: {len(TX)} sampled waves; per reflected segment k: waves with active lanes per sampled wave, "
          f"active lanes, bundle candidates, reachable spheres (per such wave)")
    for k in range(1, L + 1):
        if cnt[k, 0]:
            n = cnt[k, 0]
            print(f"  k={k}: waves {n / len(TX):.3f}  lanes {cnt[k, 1] / n:5.1f}  bundle cands {cnt[k, 2] / n:5.2f}  "
                  f"reachable {cnt[k, 3] / n:5.2f}  split-by-prev-prim cands {cnt[k, 4] / n:5.2f} (groups {cnt[k, 5] / n:4.2f})")
    tot = cnt[1:].sum(axis=0)
    print(f"  per sampled wave: bundle candidates {tot[2] / len(TX):.2f}, reachable {tot[3] / len(TX):.2f}, "
          f"split {tot[4] / len(TX):.2f} in {tot[5] / len(TX):.2f} bundles")


if __name__ == "__main__":
    main()
