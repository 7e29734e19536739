"""Generate tests/golden/ fixtures from the CPU oracle (oracle/liboracle.so).

The reference (C#/.NET 6 + OpenTK) ships no tests or golden images and cannot run in this
image, so the fixtures are produced by the oracle and cross-validated here, before being
written, by (1) the oracle's two independent drivers (all-hit reference-faithful vs
nearest-only) on every case, and (2) the independent numpy float32 emulation
(tests/emu_f32.py) on the small raw frames.

    python tests/golden/make_golden.py          # rewrites golden.json and frames_*.npy
    python tests/golden/make_golden.py --pin    # re-derives every full-size CRC with the all-hit
                                                # driver (no size cap), checks it against golden.json
                                                # and the nearest driver, writes pin_allhit.log

The all-hit driver (MODE_REFERENCE) shades every hit primitive and recurses into every mirror hit,
as RayTracer.cs:975-991 and :792-823 do; the nearest driver restates the GPU's algorithm.  With
--pin, each full-size case (C4 3840x2160 and C5 7680x4320 included) is rendered by both drivers in
row ranges (`rows=`; the reference's row-parallel loop makes rows independent) and the CRC of the
concatenated all-hit frame must equal the committed one.
"""
from __future__ import annotations

import json
import os
import sys
import time
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import emu_f32  # noqa: E402
import pyoracle  # noqa: E402
from raytracer_hip import scenes  # noqa: E402

# (case id, config, width, height): full-size frames -> CRC32 + ray counts
CRC_CASES = [
    ("REF_512", "REF", 512, 512),
    ("REF_1280x720", "REF720", 1280, 720),
    ("C1", "C1", 512, 512),
    ("C2", "C2", 1920, 1080),
    ("C3", "C3", 1920, 1080),
    ("C4", "C4", 3840, 2160),
    ("C5", "C5", 7680, 4320),
]
# small frames stored raw (and checked against the numpy emulation)
RAW_CASES = [
    ("REF_64", "REF", 64, 64),
    ("REF_128", "REF", 128, 128),
    ("C1_64", "C1", 64, 64),
    ("C2_96x54", "C2", 96, 54),
    ("C3_96x54", "C3", 96, 54),
    ("C4_64x36", "C4", 64, 36),
]


def crc(a: np.ndarray) -> str:
    return f"{zlib.crc32(np.ascontiguousarray(a, dtype=np.int32).tobytes()) & 0xFFFFFFFF:08x}"


def pin(chunk_rows: int = 256):
    """All-hit = nearest = golden.json at full size for every CRC case (no pixel cap)."""
    nthreads = min(16, os.cpu_count() or 1)
    with open(os.path.join(HERE, "golden.json")) as f:
        gold = json.load(f)["cases"]
    lines = [f"# make_golden.py --pin: all-hit driver (MODE_REFERENCE) vs nearest driver vs golden.json, "
             f"full size, {nthreads} threads, row chunks of {chunk_rows}"]
    for cid, cfg, w, h in CRC_CASES:
        sc = scenes.config(cfg).resized(w, h)
        c_ref = c_near = 0
        mism = 0
        t0 = time.time()
        for r0 in range(0, h, chunk_rows):
            r1 = min(h, r0 + chunk_rows)
            ref, _ = pyoracle.render(sc, pyoracle.MODE_REFERENCE, nthreads, rows=(r0, r1))
            near, _ = pyoracle.render(sc, pyoracle.MODE_NEAREST, nthreads, rows=(r0, r1))
            mism += int((ref != near).sum())
            c_ref = zlib.crc32(np.ascontiguousarray(ref).tobytes(), c_ref)
            c_near = zlib.crc32(np.ascontiguousarray(near).tobytes(), c_near)
        c_ref, c_near = f"{c_ref & 0xFFFFFFFF:08x}", f"{c_near & 0xFFFFFFFF:08x}"
        ok = c_ref == c_near == gold[cid]["crc32"] and mism == 0
        line = (f"{cid:14s} {w}x{h} all-hit {c_ref} nearest {c_near} golden {gold[cid]['crc32']} "
                f"mismatching pixels {mism} {'OK' if ok else 'FAIL'} ({time.time() - t0:.1f} s)")
        print(line, flush=True)
        lines.append(line)
        assert ok, line
    # the independent numpy float32 emulation (all-hit, written from the C#) on C4's scene (= C5's)
    # at a mid size, beside both drivers
    sc = scenes.config("C4").resized(384, 216)
    t0 = time.time()
    emu = emu_f32.Emu(sc).render()
    near, _ = pyoracle.render(sc, pyoracle.MODE_NEAREST, nthreads)
    ref, _ = pyoracle.render(sc, pyoracle.MODE_REFERENCE, nthreads)
    ok = np.array_equal(emu, near) and np.array_equal(emu, ref)
    line = (f"C4/C5 scene   384x216 numpy emulation {crc(emu)} nearest {crc(near)} all-hit {crc(ref)} "
            f"{'OK' if ok else 'FAIL'} ({time.time() - t0:.1f} s)")
    print(line, flush=True)
    lines.append(line)
    assert ok, line
    with open(os.path.join(HERE, "pin_allhit.log"), "w") as f:
        f.write("\n".join(lines) + "\n")


def main():
    nthreads = min(16, os.cpu_count() or 1)
    out = {"generator": "oracle/liboracle.so (nearest-hit driver)", "cases": {}}
    for cid, cfg, w, h in CRC_CASES + RAW_CASES:
        sc = scenes.config(cfg).resized(w, h)
        px, st = pyoracle.render(sc, pyoracle.MODE_NEAREST, nthreads)
        ref, _ = pyoracle.render(sc, pyoracle.MODE_REFERENCE, nthreads)  # every size, C5 included
        assert np.array_equal(ref, px), f"{cid}: all-hit vs nearest drivers differ"
        entry = {"config": cfg, "width": w, "height": h, "crc32": crc(px), "stats": st,
                 "black_fraction": float((px == 0).mean())}
        if (cid, cfg, w, h) in RAW_CASES:
            emu = emu_f32.Emu(sc).render()
            assert np.array_equal(emu, px), f"{cid}: numpy emulation differs from oracle"
            fn = f"frame_{cid}.npy"
            np.save(os.path.join(HERE, fn), px)
            entry["frame"] = fn
        out["cases"][cid] = entry
        print(cid, entry["crc32"], st, flush=True)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    pin() if "--pin" in sys.argv[1:] else main()
