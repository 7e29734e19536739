"""Per-dispatch durations of one kernel from a rocprofv3 --kernel-trace CSV, to reconcile with
bench.py's roofline.kernel_avg_ms (HIP events around the timed launches of the same process).

    python tools/trace_summary.py TRACE_DIR_OR_CSV [--kernel trace_direct_kernel] [--last 16]
                                  [--skip-last 16] [--bench bench_line.json]

Prints the average over every dispatch of the kernel (the kernel_stats.csv figure) and over the
last `--last` dispatches (the bench's timed launches: warm-up and clock-ramp launches come first),
and, with --bench, the bench line's kernel_avg_ms and their ratio.  --skip-last N leaves out the
trailing N dispatches first: bench.py's untimed second pass of the same launches (each with its
own event pair, roofline.kernel_avg_ms_launch_events), reported separately."""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default="rtk::trace_")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--skip-last", type=int, default=0)
    ap.add_argument("--bench", default="")
    a = ap.parse_args()
    fn = a.path if a.path.endswith(".csv") else glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"),
                                                           recursive=True)[0]
    rows = [r for r in csv.DictReader(open(fn)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = sorted({r["Kernel_Name"] for r in rows})
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]  # ms
    print(f"kernel(s): {'; '.join(names)}")
    if a.skip_last:
        tail = dur[-a.skip_last:]
        dur = dur[:-a.skip_last]
        print(f"trailing {len(tail)} dispatches (bench.py's untimed per-launch-event pass): average "
              f"{sum(tail) / len(tail):.4f} ms -- left out below")
    print(f"dispatches {len(dur)}: average {sum(dur) / len(dur):.4f} ms (all)")
    out = {"kernels": names, "dispatches": len(dur), "avg_ms_all": sum(dur) / len(dur)}
    if a.last:
        last = dur[-a.last:]
        out["avg_ms_last"] = sum(last) / len(last)
        print(f"last {len(last)} dispatches (the timed launches): average {out['avg_ms_last']:.4f} ms, "
              f"min {min(last):.4f}, max {max(last):.4f}")
    if a.bench:
        line = json.loads(open(a.bench).read().strip().splitlines()[-1])
        r = line["roofline"]
        print(f"bench line: kernel_avg_ms {r['kernel_avg_ms']:.4f} over {r['launches']} launches of "
              f"{r['frames_per_launch']:g} frames; ms_per_step {line['ms_per_step']:.5f}; frac {r['frac']:.5f}")
        ref = out.get("avg_ms_last", out["avg_ms_all"])
        print(f"trace / bench kernel_avg_ms = {ref / r['kernel_avg_ms']:.4f}; frac from the trace = "
              f"{r['achieved'] * r['kernel_avg_ms'] / ref / r['peak']:.5f}; kernel time per frame from the trace "
              f"{ref / r['frames_per_launch'] * 1e3:.3f} us vs ms_per_step {line['ms_per_step'] * 1e3:.3f} us")


if __name__ == "__main__":
    main()
