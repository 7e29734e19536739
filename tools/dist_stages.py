"""Per-stage timeline of the N > 1 pipeline's timed batch from a rocprofv3 kernel + HIP-runtime trace
(tools/dist_trace.sh: bench.py --dist-path --rank0-codec --steps 20, world 1, C2).

The run ends with: warm-up batches, the timed batch, then an untimed second pass of the same batch
(bench.py's launch-event cross-check).  Each batch is one fused trace launch (rt_render_bands_tiles),
the codec's finish (chunk totals + copy), RCCL's size all_reduce and gather, and rank 0's decode.  The
timed batch is the last-but-one trace launch of the 20-frame shape; its stages are listed in start
order with their durations and the idle gaps between them on the GPU."""
import csv
import glob
import os
import sys


def short(name):
    for key, lab in (("trace_direct_kernel", "trace (fused encoder)"), ("trace_bundle_kernel", "trace (fused encoder)"),
                     ("chunk_totals", "finish: chunk totals"), ("encode_copy", "finish: copy"),
                     ("decode_tiles", "decode"), ("AllReduce", "RCCL all_reduce"), ("Gather", "RCCL gather"),
                     ("ncclDevKernel", "RCCL kernel"), ("elementwise", "torch elementwise"), ("copyBuffer", "runtime copy"),
                     ("fillBuffer", "runtime fill")):
        if key in name:
            return lab
    return name[:60]


def main():
    d = sys.argv[1]
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = sorted(csv.DictReader(open(kf)), key=lambda r: int(r["Start_Timestamp"]))
    traces = [i for i, r in enumerate(ks) if "trace_" in r["Kernel_Name"] and "_kernel" in r["Kernel_Name"]]
    # the timed batch: the last-but-one trace launch; its window runs to the next trace launch
    a, b = traces[-2], traces[-1]
    win = ks[a:b]
    t0 = int(win[0]["Start_Timestamp"])
    print(f"# timed batch: kernels {a}..{b - 1} of {len(ks)} (trace launches in the run: {len(traces)})")
    print(f"{'stage':34s} {'start us':>9s} {'dur us':>9s} {'gap before us':>14s}")
    last_end = t0
    busy = 0
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, s - last_end)
        print(f"{short(r['Kernel_Name']):34s} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f} {gap / 1e3:14.1f}")
        busy += e - s
        last_end = max(last_end, e)
    span = last_end - t0
    print(f"# window {span / 1e3:.1f} us: kernels busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us "
          f"({span / 1e3 / 20:.2f} us per frame of 20)")
    hf = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    if hf:
        api = [r for r in csv.DictReader(open(hf[0]))
               if t0 - 200_000 <= int(r["Start_Timestamp"]) <= last_end + 200_000]
        tot = {}
        for r in api:
            tot.setdefault(r["Function"], [0, 0])
            tot[r["Function"]][0] += 1
            tot[r["Function"]][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print("# HIP API calls from 200 us before the window to 200 us after (count, host us)")
        for f, (n, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:15]:
            print(f"  {f:40s} {n:6d} {t / 1e3:10.1f}")


if __name__ == "__main__":
    main()
