"""rt_count_work of several library builds side by side (executed shadow rays / sphere tests per frame).
    python tools/work_compare.py --configs C4 C5 LIB_A LIB_B ..."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--configs", nargs="+", default=["C4", "C5"])
    a = ap.parse_args()
    for n in a.configs:
        for lib in a.libs:
            code = ("import sys, json; sys.path.insert(0, %r); from raytracer_hip import abi, Context, scenes; "
                    "abi.LIB_PATH = %r; sc = scenes.config(%r); c = Context(1); c.set_scene(sc); "
                    "print(json.dumps(c.count_work(sc.width, sc.height)))") % (
                os.path.join(ROOT, "uu-infogr-raytracer_amd"), os.path.abspath(lib), n)
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
            if r.returncode:
                raise SystemExit(r.stderr[-2000:])
            w = json.loads(r.stdout.strip().splitlines()[-1])
            print(f"{n} {os.path.basename(lib):36s} shadow rays {w['shadow_rays']:,} run {w['shadow_rays_run']:,}  "
                  f"sphere tests run {w['sphere_tests_run']:,}", flush=True)


if __name__ == "__main__":
    main()
