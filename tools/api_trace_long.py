"""Long HIP API calls in a rocprofv3 --hip-runtime-trace CSV (the deep Tick probe's stalls): every call over
--min-us, with the calls just before it on the same thread and the kernels / copies that ran during it.

    python tools/api_trace_long.py gpurun_out/r06/tick_trace [--min-us 1000]
"""
import argparse
import csv
import glob
import os
from collections import Counter


def rows(d, suffix):
    out = []
    for fn in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        out += list(csv.DictReader(open(fn)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=1000.0)
    a = ap.parse_args()
    api = rows(a.dir, "hip_api_trace.csv")
    kern = rows(a.dir, "kernel_trace.csv")
    copies = rows(a.dir, "memory_copy_trace.csv")
    for r in api:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    api.sort(key=lambda r: r["t0"])
    print(f"{len(api)} HIP API calls, {len(kern)} kernels, {len(copies)} copies")
    tot = Counter()
    for r in api:
        tot[r["Function"]] += r["t1"] - r["t0"]
    print("API time by function (top 12, ms):", ", ".join(f"{f} {t / 1e6:.2f}" for f, t in tot.most_common(12)))
    for i, r in enumerate(api):
        dt = (r["t1"] - r["t0"]) / 1e3
        if dt < a.min_us:
            continue
        prev = [p for p in api[max(0, i - 12):i] if p["Thread_Id"] == r["Thread_Id"]][-6:]
        during_k = [k for k in kern if int(k["Start_Timestamp"]) < r["t1"] and int(k["End_Timestamp"]) > r["t0"]]
        during_c = [c for c in copies if int(c["Start_Timestamp"]) < r["t1"] and int(c["End_Timestamp"]) > r["t0"]]
        print(f"\n{r['Function']} {dt:.1f} us (thread {r['Thread_Id']}), after: "
              + " | ".join(f"{p['Function']} {(p['t1'] - p['t0']) / 1e3:.1f}" for p in prev))
        kb = sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in during_k) / 1e3
        cb = sum(int(c["End_Timestamp"]) - int(c["Start_Timestamp"]) for c in during_c) / 1e3
        print(f"  during it: {len(during_k)} kernels ({kb:.1f} us busy), {len(during_c)} copies ({cb:.1f} us busy)")
        if during_k:
            first = min(int(k["Start_Timestamp"]) for k in during_k)
            print(f"  first kernel during it starts {(first - r['t0']) / 1e3:.1f} us after the call;"
                  f" kernels: {Counter(k['Kernel_Name'][:60] for k in during_k).most_common(3)}")


if __name__ == "__main__":
    main()
