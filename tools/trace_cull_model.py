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
    for count in range(sc.recursion_limit + 2):
        if count == sc.recursion_limit + 1:
            # terminal segment (rt_kernel.hip trace_tile_bundle): only lanes whose nearest plane lies beyond
            # 0.01 test the spheres
            with np.errstate(divide="ignore", invalid="ignore"):
                tp = (np.einsum("pk,pk->p", PC, PN)[None] - o @ PN.T) / (d @ PN.T)
            tp = np.where(tp > 0, tp, np.inf).min(axis=1)
            segs.append((o.copy(), d.copy(), active & np.isfinite(tp) & (tp - 0.01 > 0), prev.copy()))
            break
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


def clusters(C, r, size):
    """Spatial clusters of at most `size` spheres (median splits along the widest axis of the centres), each
    with a bounding sphere (centre: the middle of its centres' box; radius: max |c_i - Cc| + r_i).  Returns
    (member masks (K, S) bool, centres (K, 3), radii (K,))."""
    groups, todo = [], [np.arange(len(C))]
    while todo:
        g = todo.pop()
        if len(g) <= size:
            groups.append(g)
            continue
        ax = np.argmax(C[g].max(axis=0) - C[g].min(axis=0))
        g = g[np.argsort(C[g, ax], kind="stable")]
        todo += [g[:len(g) // 2], g[len(g) // 2:]]
    M = np.zeros((len(groups), len(C)), bool)
    Cc = np.zeros((len(groups), 3))
    Rc = np.zeros(len(groups))
    for i, g in enumerate(groups):
        M[i, g] = True
        Cc[i] = (C[g].max(axis=0) + C[g].min(axis=0)) / 2
        Rc[i] = (np.linalg.norm(C[g] - Cc[i], axis=1) + r[g]).max()
    return M, Cc, Rc


def cluster_union(o, d, M, Cc, Rc):
    """Per-lane cluster pre-cull: lane l keeps cluster j unless its ray line misses the bounding sphere or the
    sphere lies wholly behind its origin (2^-8 margins, as cull_mask); the wave takes the union of the kept
    clusters' members.  -> candidate mask (S,), clusters kept by some lane."""
    w = Cc[None] - o[:, None, :]                                   # (k, K, 3)
    a = np.einsum("kj,kj->k", d, d)[:, None]
    wd = np.einsum("kcj,kj->kc", w, d)
    ww = np.einsum("kcj,kcj->kc", w, w)
    R = Rc[None] * (1 + 2 ** -8) + 2 ** -8 * np.sqrt(ww)
    line = ww * a - wd * wd > R * R * a
    behind = wd < -R * np.sqrt(a)
    keep = ~(line | behind)
    kc = keep.any(axis=0)
    return M[kc].any(axis=0), kc.sum()


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
    cnt = np.zeros((L + 2, 6))  # waves, active lanes, bundle candidates, reachable, split by previous primitive, groups
    sizes = (2, 4, 8)
    CL = {z: clusters(C, np.sqrt(r2), z) for z in sizes}
    ccnt = np.zeros((L + 2, len(sizes), 4))  # per cluster size: union, union & bundle, clusters kept, cluster tests
    nok = np.zeros((L + 2, 2 + len(sizes)))  # bundles that allow no culling (cone >= 0.5): count, reachable, union per z
    thr = (8, 16, 24)
    okb = np.zeros((len(thr), 3, len(sizes)))  # usable bundles with > thr candidates: count, candidates, & clusters
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
                bm = bundle_cull(o[w][m], d[w][m], C, rr)
                cnt_reach = reachable(o[w][m], d[w][m], C, r2).sum()
                cnt[k] += (1, m.sum(), bm.sum(), cnt_reach,
                           split, 1 + g2.any())
                unusable = bm.all()  # (the in-kernel !B.ok: every sphere a candidate)
                if unusable:
                    nok[k, :2] += (1, cnt_reach)
                for zi, z in enumerate(sizes):
                    um, kept = cluster_union(o[w][m], d[w][m], *CL[z])
                    ccnt[k, zi] += (um.sum(), (um & bm).sum(), kept, len(CL[z][2]))
                    if unusable:
                        nok[k, 2 + zi] += um.sum()
                    else:
                        for ti, tv in enumerate(thr):
                            if bm.sum() > tv:
                                okb[ti, :, zi] += (1, bm.sum(), (um & bm).sum())
    print(f"# {sc.name}: {len(TX)} sampled waves; per reflected segment k: waves with active lanes per sampled wave, "
          f"active lanes, bundle candidates, reachable spheres (per such wave)")
    for k in range(1, L + 2):
        if cnt[k, 0]:
            n = cnt[k, 0]
            print(f"  k={k}{'T' if k == L + 1 else ' '}: waves {n / len(TX):.3f}  lanes {cnt[k, 1] / n:5.1f}  bundle cands "
                  f"{cnt[k, 2] / n:5.2f}  reachable {cnt[k, 3] / n:5.2f}  split-by-prev-prim cands {cnt[k, 4] / n:5.2f} "
                  f"(groups {cnt[k, 5] / n:4.2f})")
            print("         per-lane cluster pre-cull (clusters of <= z spheres): " + "  ".join(
                f"z={z}: union {ccnt[k, zi, 0] / n:5.2f} & bundle {ccnt[k, zi, 1] / n:5.2f} "
                f"(kept {ccnt[k, zi, 2] / n:4.1f}/{ccnt[k, zi, 3] / n:.0f})" for zi, z in enumerate(sizes)))
    tot = cnt[1:].sum(axis=0)
    print(f"  per sampled wave (k = 1..{L + 1}, T = the terminal segment): bundle candidates {tot[2] / len(TX):.2f}, "
          f"reachable {tot[3] / len(TX):.2f}, split {tot[4] / len(TX):.2f} in {tot[5] / len(TX):.2f} bundles")
    ct = ccnt[1:].sum(axis=0)
    print("  per sampled wave, cluster pre-cull AND bundle: " + "  ".join(
        f"z={z}: {ct[zi, 1] / len(TX):.2f} candidates + {ct[zi, 3] / len(TX):.1f} cluster tests" for zi, z in enumerate(sizes)))
    S = len(C)
    print(f"  bundles that allow no culling (all {S} spheres tested today), per sampled wave and k: " + "  ".join(
        f"k={k}: {nok[k, 0] / len(TX):.3f} (reach {nok[k, 1] / max(nok[k, 0], 1):.1f}, union " +
        "/".join(f"{nok[k, 2 + zi] / max(nok[k, 0], 1):.1f}" for zi in range(len(sizes))) + ")"
        for k in range(1, L + 2) if nok[k, 0]))
    tn = nok.sum(axis=0)
    for zi, z in enumerate(sizes):
        K = len(CL[z][2])
        # VALU per lane, rough: an exact sphere test ~22 ops (b, c, disc, candidate, take), a cluster test ~14
        save = tn[0] * S * 22 - tn[0] * K * 14 - tn[2 + zi] * 22
        print(f"  pre-cull on those bundles only, z={z} ({K} clusters): candidates {tn[0] * S / len(TX):.2f} -> "
              f"{tn[2 + zi] / len(TX):.2f} per sampled wave + {tn[0] * K / len(TX):.2f} cluster tests; "
              f"~{save / len(TX):.0f} VALU ops per wave saved (of ~2,075 per C4 wave, r05 PMC)")
    for ti, tv in enumerate(thr):
        print(f"  usable bundles with > {tv} candidates: {okb[ti, 0, 0] / len(TX):.3f} per sampled wave, "
              f"{okb[ti, 1, 0] / len(TX):.2f} candidates -> & clusters " +
              " / ".join(f"z={z}: {okb[ti, 2, zi] / len(TX):.2f} (+{okb[ti, 0, 0] * len(CL[z][2]) / len(TX):.2f} cluster tests)"
                         for zi, z in enumerate(sizes)))
    for k0 in (2, 3, 4):  # pre-cull only from segment k0 on (a wave-uniform gate on the segment index)
        b = cnt[1:k0, 2].sum() + sum(ccnt[k0:, zi, 1].sum() for zi in [1])
        print(f"  pre-cull (z=8) from k={k0}: candidates {b / len(TX):.2f}, cluster tests {ccnt[k0:, 1, 3].sum() / len(TX):.2f}")


if __name__ == "__main__":
    main()
