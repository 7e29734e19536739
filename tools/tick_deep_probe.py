"""r06: the queued async Tick's slow first timed run and the 1080p Tick chunk sweep
(VERDICT r05 item 5), on one GPU.

    python tools/tick_deep_probe.py deep  [--config C3] [--runs 6]
    python tools/tick_deep_probe.py chunks [--configs C2 C3]

deep: the bench's tick_rates sequence (bench.py) up to the deep shape, then `runs` runs of the deep shape
(n frames queued into n registered buffers, one rt_wait), each with the host time of every rt_render_async
call and of the closing rt_wait -- a call that blocks shows as a long entry.  Variants: `fresh` (the deep
shape first, right after registration), `touched` (every buffer written by a synchronous Tick first).
chunks: synchronous rt_render at RT_TICK_CHUNKS = 1..4 (median of 5 runs of 20 frames, 2 interleaved passes).
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def deep_runs(ctx, W, H, hosts, runs, label):
    label = f"{label:18s}"
    n = len(hosts)
    for r in range(runs):
        calls = []
        t0 = time.perf_counter()
        for k in range(n):
            a = time.perf_counter()
            ctx.render_async(W, H, hosts[k])
            calls.append(time.perf_counter() - a)
        a = time.perf_counter()
        ctx.wait()
        tw = time.perf_counter() - a
        dt = time.perf_counter() - t0
        top = sorted(range(n), key=lambda i: -calls[i])[:3]
        print(f"{label} run {r}: {n / dt:8.1f} fps  total {dt * 1e3:7.2f} ms  calls sum {sum(calls) * 1e3:6.2f} ms "
              f"(max {max(calls) * 1e6:7.1f} us at frames {top}: {[round(calls[i] * 1e6) for i in top]})  "
              f"wait {tw * 1e3:6.2f} ms", flush=True)


def deep(args):
    import torch
    from raytracer_hip import Context, scenes
    sc = scenes.config(args.config)
    W, H, n = sc.width, sc.height, 20
    torch.cuda.set_device(0)
    for variant, inflight, mode in [(v, q, m) for m in args.modes for q in args.inflight for v in args.variants]:
        os.environ["RT_TICK_INFLIGHT"] = str(inflight)  # (read at rt_create)
        os.environ["RT_TICK_ASYNC"] = mode
        label = f"{variant} q{inflight} {mode}"
        with Context(1) as ctx:
            ctx.set_scene(sc)
            ctx.set_counting(False)
            hosts = [np.zeros(W * H, dtype=np.int32) for _ in range(n)]
            for hb in hosts:
                ctx.register_host(hb)
            if variant == "bench":  # bench.py tick_rates up to the deep shape (warm + 3 runs each)
                dev = torch.empty(W * H, dtype=torch.int32, device="cuda")
                st = torch.cuda.current_stream().cuda_stream
                for frames in [200] * 4 + [20] * 4:
                    for _ in range(frames):
                        ctx.render_device(W, H, dev.data_ptr(), st)
                    torch.cuda.synchronize()
                for _ in range(4 * n):
                    ctx.render(W, H, hosts[0])
                for _ in range(4):
                    for k in range(n):
                        ctx.render_async(W, H, hosts[k % 2])
                        if k % 2:
                            ctx.wait()
                    ctx.wait()
            elif variant == "touched":  # every buffer once by the synchronous Tick
                for hb in hosts:
                    ctx.render(W, H, hb)
            t = time.perf_counter()
            deep_runs(ctx, W, H, hosts, args.runs, label)
            print(f"{label:10s} ({(time.perf_counter() - t) * 1e3:.1f} ms for {args.runs} runs)", flush=True)
            for hb in hosts:
                ctx.unregister_host(hb)


def chunks(args):
    from raytracer_hip import Context, scenes
    for name in args.configs:
        sc = scenes.config(name)
        W, H, n = sc.width, sc.height, 20
        with Context(1) as ctx:
            ctx.set_scene(sc)
            ctx.set_counting(False)
            buf = np.zeros(W * H, dtype=np.int32)
            ctx.register_host(buf)
            res = {}
            for _ in range(2):
                for k in (1, 2, 3, 4):
                    os.environ["RT_TICK_CHUNKS"] = str(k)
                    for _ in range(n):
                        ctx.render(W, H, buf)  # warm (and a new chunk shape)
                    rates = []
                    for _ in range(5):
                        t = time.perf_counter()
                        for _ in range(n):
                            ctx.render(W, H, buf)
                        rates.append(n / (time.perf_counter() - t))
                    res.setdefault(k, []).append(sorted(rates)[2])
            os.environ.pop("RT_TICK_CHUNKS", None)
            for k, v in res.items():
                print(f"{name} sync RT_TICK_CHUNKS={k}: {' '.join(f'{x:7.1f}' for x in v)} fps "
                      f"({W * H * 4 * max(v) / 1e9:.1f} GB/s of frame)", flush=True)
            ctx.unregister_host(buf)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["deep", "chunks"])
    ap.add_argument("--config", default="C3")
    ap.add_argument("--configs", nargs="+", default=["C2", "C3"])
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--variants", nargs="+", default=["bench", "fresh", "touched"])
    ap.add_argument("--lib", default="", help="library build to load instead of the in-tree one")
    ap.add_argument("--inflight", nargs="+", type=int, default=[0], help="RT_TICK_INFLIGHT values (0: no bound)")
    ap.add_argument("--modes", nargs="+", default=["stream"], help="RT_TICK_ASYNC values (stream: copy engine)")
    args = ap.parse_args()
    if args.lib:
        from raytracer_hip import abi
        abi.LIB_PATH = os.path.abspath(args.lib)
    deep(args) if args.what == "deep" else chunks(args)


if __name__ == "__main__":
    main()
