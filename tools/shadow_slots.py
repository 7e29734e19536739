"""Where the bundle kernel's idle shadow-test lane slots are (C4/C5): rt_count_work with the
RT_SHADOW_CAT=1 diagnostic build counts the shadow-test slots of one category (RT_DIAG_SEL), per
fold level.  GPU box:
    make -C uu-infogr-raytracer_amd/csrc variant NAME=shcat VFLAGS=-DRT_SHADOW_CAT=1
    python tools/shadow_slots.py --configs C4 C5"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CATS = ["useful", "needed, blocked", "diffuse, not needed", "active, not diffuse", "no record"]


def count(lib, name, sel):
    code = ("import sys, json; sys.path.insert(0, %r); from raytracer_hip import abi, Context, scenes; "
            "abi.LIB_PATH = %r; sc = scenes.config(%r); c = Context(1); c.set_scene(sc); "
            "print(json.dumps(c.count_work(sc.width, sc.height)))") % (
        os.path.join(ROOT, "uu-infogr-raytracer_amd"), lib, name)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, RT_DIAG_SEL=str(sel)))
    if r.returncode:
        raise SystemExit(r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])["sphere_tests_run"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["C4"])
    ap.add_argument("--levels", type=int, default=6)
    ap.add_argument("--lib", default=os.path.join(ROOT, "uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_shcat.so"))
    a = ap.parse_args()
    for n in a.configs:
        tab = {}
        for c in range(1, 6):
            tab[c] = [count(a.lib, n, 16 * c + lv + 1) for lv in range(a.levels)]
        tot = sum(sum(v) for v in tab.values())
        print(f"{n}: shadow-test lane slots per frame {tot:,} (useful {sum(tab[1]) / tot:.3f})", flush=True)
        print("  level " + " ".join(f"{lv:>13d}" for lv in range(a.levels)) + "        total", flush=True)
        for c in range(1, 6):
            print(f"  {CATS[c - 1]:22s}" + " ".join(f"{v:13,d}" for v in tab[c]) + f" {sum(tab[c]):13,d}", flush=True)
        lvl_tot = [sum(tab[c][lv] for c in tab) for lv in range(a.levels)]
        print(f"  {'all':22s}" + " ".join(f"{v:13,d}" for v in lvl_tot), flush=True)
        # overlap of the lights' candidate sets (per wave and shaded level): sum over lights vs union
        per = [count(a.lib, n, 16 * 6 + lv + 1) for lv in range(a.levels)]
        uni = [count(a.lib, n, 16 * 7 + lv + 1) for lv in range(a.levels)]
        print(f"  {'cands, sum of lights':22s}" + " ".join(f"{v:13,d}" for v in per) + f" {sum(per):13,d}", flush=True)
        print(f"  {'cands, union':22s}" + " ".join(f"{v:13,d}" for v in uni) + f" {sum(uni):13,d}", flush=True)


if __name__ == "__main__":
    main()
