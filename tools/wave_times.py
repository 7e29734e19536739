"""Where a lone frame's launch spends its time (tools/build_wave_times.sh builds the probe library): every
direct- and bundle-kernel wave records its start (s_memrealtime, 100 MHz), duration and HW_ID/XCC_ID.  Prints the ramp
(when the waves start), the tail (when the CUs go idle), the slowest tiles and a coarse map of wave durations.
    python tools/wave_times.py --lib uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_wt.so --config C2 [--batch 1]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))
TICK_US = 0.01  # s_memrealtime: 100 MHz


def pct(a, q):
    return float(np.percentile(a, q)) if len(a) else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--lib", required=True)
    ap.add_argument("--batch", type=int, default=1, help="frames per launch (1: the single-frame launch)")
    ap.add_argument("--reps", type=int, default=5, help="launches analysed (each the last of a back-to-back run)")
    ap.add_argument("--map", action="store_true", help="print a coarse map of wave durations")
    ap.add_argument("--save", default="", help="write the last launch's per-tile start / duration (us) to this .npz")
    a = ap.parse_args()
    import torch
    from raytracer_hip import Context, abi, scenes
    abi.LIB_PATH = os.path.abspath(a.lib)
    sc = scenes.config(a.config)
    W, H = sc.width, sc.height
    ctx = Context(1)
    ctx.set_scene(sc)
    lib = C.CDLL(abi.LIB_PATH)
    lib.rt_debug_wave_times.argtypes = [C.c_void_p, C.c_size_t]
    tx, ty = (W + 7) // 8, (H + 7) // 8
    n = tx * ty * a.batch
    assert n <= 1 << 20
    st = torch.cuda.current_stream()
    big = torch.empty(a.batch * W * H, dtype=torch.int32, device="cuda")

    def launch():
        if a.batch > 1:
            ctx.render_bands_batch(W, H, 8, 0, 1, a.batch, big.data_ptr(), W * H * 4, abi.RT_BANDS_FRAME, st.cuda_stream)
        else:
            ctx.render_device(W, H, big.data_ptr(), st.cuda_stream)
    rows = []
    for rep in range(a.reps):
        for _ in range(30):
            launch()
        torch.cuda.synchronize()
        buf = np.zeros((1 << 20, 4), dtype=np.uint32)
        assert lib.rt_debug_wave_times(buf.ctypes.data, buf.nbytes) == 0
        r = buf[:n]
        start = r[:, 0].astype(np.int64)  # RTC low 32 bits: unwrap (a launch lasts far less than 2^31 ticks)
        if start.max() - start.min() > (1 << 31):
            start = np.where(start < (1 << 31), start + (1 << 32), start)
        start -= start.min()
        dur = r[:, 2].astype(np.int64)
        cyc = r[:, 1].astype(np.int64)  # shader-clock cycles of the wave (s_memtime)
        mhz = cyc / np.maximum(dur, 1) * 100.0  # RTC ticks at 100 MHz
        end = start + dur
        span = end.max()
        hw, xcc = r[:, 3] & 0xFFFFFF, r[:, 3] >> 24
        cu = (xcc.astype(np.int64) << 16) | ((hw >> 13) & 0x7).astype(np.int64) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 0xF)
        ncu = len(np.unique(cu))
        last_end = {}
        for c, e in zip(cu, end):
            last_end[c] = max(last_end.get(c, 0), e)
        idle_tail = float(np.mean([span - e for e in last_end.values()]))
        rows.append(dict(span=span * TICK_US, start50=pct(start, 50) * TICK_US, start90=pct(start, 90) * TICK_US,
                         start100=start.max() * TICK_US, end10=pct(end, 10) * TICK_US, end50=pct(end, 50) * TICK_US,
                         end90=pct(end, 90) * TICK_US, end99=pct(end, 99) * TICK_US, dur50=pct(dur, 50) * TICK_US,
                         dur99=pct(dur, 99) * TICK_US, durmax=dur.max() * TICK_US, cus=ncu, idle_tail=idle_tail * TICK_US,
                         work=float(dur.sum()) * TICK_US,
                         mhz=float(np.sum(cyc) / max(np.sum(dur), 1) * 100.0)))
        if rep == a.reps - 1 and a.save:
            np.savez(a.save, start=start * TICK_US, dur=dur * TICK_US, cyc=cyc, tiles_x=tx, tiles_y=ty)
        if rep == a.reps - 1:
            order = np.argsort(-end)[:12]
            print(f"# {a.config} {W}x{H} batch={a.batch}: {n} waves on {ncu} CUs; the 12 last to finish "
                  f"(tile x, y, frame: start, duration us):")
            for i in order:
                f, t = divmod(int(i), tx * ty)
                print(f"   ({t % tx:3d},{t // tx:3d},{f}) start {start[i] * TICK_US:7.2f} dur {dur[i] * TICK_US:6.2f}")
            # time series: resident waves (whole chip) per 1 us
            step = 100 if span < 20000 else 1000  # 1 us, or 10 us for long launches (C4/C5)
            edges = np.arange(0, span + step, step)
            res = [(int(((start <= t) & (end > t)).sum())) for t in edges]
            print(f"# resident waves per {step // 100} us:", " ".join(str(x) for x in res))
            # shader clock seen by the waves (cycles / RTC time), per frame and per 100 us of start time
            per = tx * ty
            for f in range(a.batch):
                sl = slice(f * per, (f + 1) * per)
                print(f"# frame {f}: wave-us {dur[sl].sum() * TICK_US:.0f}, clock {cyc[sl].sum() / max(dur[sl].sum(), 1) * 100:.0f} MHz, "
                      f"cycles {cyc[sl].sum() / 1e6:.1f} M")
            bucket = 10000  # 100 us
            line = []
            for b0 in range(0, int(span) + 1, bucket):
                k = (start >= b0) & (start < b0 + bucket)
                if k.sum() > 100:
                    line.append(f"{b0 // 100}:{cyc[k].sum() / max(dur[k].sum(), 1) * 100:.0f}")
            print("# clock (MHz) of the waves starting in each 100 us:", " ".join(line))
            if a.map:
                d = dur[: tx * ty].reshape(ty, tx).astype(float) * TICK_US
                by, bx = max(1, ty // 34), max(1, tx // 60)
                dm = d[: ty // by * by, : tx // bx * bx].reshape(ty // by, by, tx // bx, bx).mean(axis=(1, 3))
                q = np.quantile(dm, [0.2, 0.4, 0.6, 0.8, 0.95])
                chars = " .:-=#"
                print(f"# mean wave duration map ({bx}x{by} tiles per cell; quantile cuts {np.round(q, 2).tolist()} us)")
                for row in dm:
                    print("   |" + "".join(chars[int(np.searchsorted(q, v))] for v in row) + "|")
    keys = list(rows[0])
    med = {k: float(np.median([r[k] for r in rows])) for k in keys}
    print(f"# medians over {a.reps} launches (us): " + ", ".join(f"{k} {med[k]:.2f}" for k in keys))
    print(f"# wave-us per frame {med['work'] / a.batch:.1f}; span per frame {med['span'] / a.batch:.2f} us; "
          f"mean CU idle after its last wave {med['idle_tail']:.2f} us")


if __name__ == "__main__":
    main()
