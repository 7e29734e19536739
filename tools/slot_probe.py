"""Lane utilisation of the exact sphere tests (the bound on what secondary-ray compaction could
recover): rt_count_work's executed sphere tests with the in-tree library (lanes whose result is
used) and with the RT_SLOT_TALLY build (every lane slot a test occupied, idle lanes included --
the bundle kernel's idle lanes trace copies of an active lane's ray) -- RT_SLOT_TALLY=1 every
test, =2 the nearest-hit tests only (the shadow loops count their useful lanes), which splits
the idle slots between nearest-hit and shadow tests.  GPU box:
    make -C uu-infogr-raytracer_amd/csrc variant NAME=slots VFLAGS=-DRT_SLOT_TALLY=1
    make -C uu-infogr-raytracer_amd/csrc variant NAME=slots2 VFLAGS=-DRT_SLOT_TALLY=2
    python tools/slot_probe.py --configs C2 C3 C4 C5"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def counts(lib, names):
    import subprocess
    code = ("import sys, json; sys.path.insert(0, %r); from raytracer_hip import abi, Context, scenes; "
            "abi.LIB_PATH = %r; out = {}\n"
            "for n in %r:\n"
            "    sc = scenes.config(n); c = Context(1); c.set_scene(sc); out[n] = c.count_work(sc.width, sc.height); c.close()\n"
            "print(json.dumps(out))") % (os.path.join(ROOT, "uu-infogr-raytracer_amd"), lib, names)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if r.returncode:
        raise SystemExit(r.stderr[-2000:])
    import json
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["C2", "C3", "C4", "C5"])
    ap.add_argument("--slots-lib", default=os.path.join(ROOT, "uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_slots.so"))
    ap.add_argument("--slots2-lib", default=os.path.join(ROOT, "uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_slots2.so"))
    ap.add_argument("--base-lib", default=os.path.join(ROOT, "uu-infogr-raytracer_amd/lib/libraytracer_hip.so"),
                    help="the timed build whose executed (useful) tests are counted")
    a = ap.parse_args()
    base = counts(a.base_lib, a.configs)
    slots = counts(a.slots_lib, a.configs)
    slots2 = counts(a.slots2_lib, a.configs)
    for n in a.configs:
        u, s, s2 = base[n]["sphere_tests_run"], slots[n]["sphere_tests_run"], slots2[n]["sphere_tests_run"]
        print(f"{n}: exact sphere tests per frame: useful lanes {u:,}, lane slots {s:,} -> useful {u / s:.3f}; "
              f"idle slots in nearest-hit tests {s2 - u:,}, in shadow tests {s - s2:,}")


if __name__ == "__main__":
    main()
