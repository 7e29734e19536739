"""Back-to-back single-frame launches (one trace dispatch per frame) from a rocprofv3 --kernel-trace:
average dispatch duration and the idle gap between the end of one trace dispatch and the start
of the next -- what separates the interactive one-frame-per-Tick rate from the batched one.

    python tools/single_gap.py TRACE_DIR_OR_CSV [--kernel rtk::trace_] [--last 200]"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default="rtk::trace_")
    ap.add_argument("--last", type=int, default=200)
    a = ap.parse_args()
    fn = a.path if a.path.endswith(".csv") else glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"),
                                                           recursive=True)[0]
    rows = [r for r in csv.DictReader(open(fn)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.last:]
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    dur = sorted((e - s) / 1e3 for s, e in zip(st, en))
    gap = sorted((st[i + 1] - en[i]) / 1e3 for i in range(len(rows) - 1))
    per = (en[-1] - st[0]) / 1e3 / len(rows)
    med = lambda x: x[len(x) // 2]  # noqa: E731
    print(f"{len(rows)} dispatches ({rows[0]['Kernel_Name'][:60]}): duration median {med(dur):.2f} us "
          f"(min {dur[0]:.2f}, max {dur[-1]:.2f}); gap end->next start median {med(gap):.2f} us "
          f"(min {gap[0]:.2f}, max {gap[-1]:.2f}); period {per:.2f} us per frame")


if __name__ == "__main__":
    main()
