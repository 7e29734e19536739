"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh output): per-dispatch average of every
counter for one kernel.  HBM traffic per launch follows MI355X_MICROARCH.md 'HBM':
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide
coalesced reads, so it is doubled; WRITE_SIZE is taken as is.

    python tools/pmc_summary.py gpurun_out/pmc_C2 [kernel-substring] [--json out.json --config C2 --world 1
                                                                      --frames-per-launch 16]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d, kernel="rtk::trace_"):
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    files = glob.glob(os.path.join(d, "p*", "*counter_collection.csv")) + glob.glob(os.path.join(d, "*counter_collection.csv"))
    for fn in sorted(files):
        for row in csv.DictReader(open(fn)):
            if kernel not in row["Kernel_Name"]:
                continue
            key = (fn, row["Dispatch_Id"])
            vals[row["Counter_Name"]][key] += float(row["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in vals.items() if v}


def main():
    d = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "rtk::trace_"
    s = summarise(d, kernel)
    for k in sorted(s):
        print(f"{k:32s} {s[k]:,.1f}")
    fetch = s.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = s.get("WRITE_SIZE", 0.0) * 1024
    print(f"{'HBM bytes/launch (corrected)':32s} {fetch + write:,.0f}  (fetch x2 {fetch:,.0f} + write {write:,.0f})")
    if "SQ_THREAD_CYCLES_VALU" in s and "SQ_ACTIVE_INST_VALU" in s:
        print(f"{'VALU lane utilisation':32s} {s['SQ_THREAD_CYCLES_VALU'] / (64 * s['SQ_ACTIVE_INST_VALU']):.3f}")
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        cfg = sys.argv[sys.argv.index("--config") + 1]
        world = sys.argv[sys.argv.index("--world") + 1] if "--world" in sys.argv else "1"
        try:
            data = json.load(open(out))
        except (OSError, ValueError):
            data = {}
        fpl = int(sys.argv[sys.argv.index("--frames-per-launch") + 1]) if "--frames-per-launch" in sys.argv else 1
        data.setdefault(cfg, {})[world] = {
            "hbm_bytes_per_launch": fetch + write, "frames_per_launch": fpl, "fetch_size_kib": s.get("FETCH_SIZE"),
            "write_size_kib": s.get("WRITE_SIZE"), "counters": s,
            "method": "rocprofv3 --pmc, one pass per counter group; FETCH_SIZE x2 (gfx950), KiB -> bytes"}
        json.dump(data, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
