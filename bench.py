#!/usr/bin/env python3
"""bench.py -- the hot path of BASELINE.json on MI355X.

One step = one frame of the per-pixel trace (RayTracer.Tick, Raytracer/RayTracer.cs:886-935)
on the configuration named by --config (default C3 = BASELINE.json configs[2], the north-star's
target config: 1920x1080, 8 spheres + 1 plane, 2 lights, recursive mirror reflections depth 4),
with the scene resident in HBM and the frame written to HBM.

N = 1: the timed frames run as balanced launches of up to 64 frames (rt_render_bands_batch),
one launch in flight, back to back on one stream: HIP events around the timed region / launches
give roofline.kernel_avg_ms (which rocprofv3's kernel trace of the same command reproduces); an
untimed second pass times each launch with its own event pair (kernel_avg_ms_launch_events).  C2 (configs[1]: depth 1,
1 light), C4 and C5 are measured in the same run ("also"), and the plugin path's Tick() (rt_render / rt_render_async
into registered host memory, PCIe included) for C2-C5 under tick_by_config.

N > 1 (`--gpus N`: one process per GPU; started here through torch.distributed.run when no
launcher set WORLD_SIZE): the frame is split into interleaved 8-row bands, band b on rank
b % N, and the band sets are gathered to rank 0 over RCCL (torch.distributed backend "nccl"
is RCCL on ROCm) -- strong scaling of a fixed frame.  Then rank 0 runs the plugin path's own multi-GPU
Tick() in one process (Context(N): every device hands its bands to the host frame over its own PCIe
link), reported under plugin_tick.

Prints ONE JSON line (rank 0).  Rays = primary + reflected + shadow rays of the visible
(nearest-hit) path, counted by the kernel itself (rt_get_stats); `work_per_frame` sets the
tests the kernels actually executed beside those nominal counts.
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "uu-infogr-raytracer_amd")
sys.path.insert(0, PKG)

METRIC = "Mray/s (primary+shadow+reflect) and fps at 1920×1080, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 78.64         # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz, one non-FMA f32 op per lane
OPS_PER_SPHERE_TEST = 24       # miss-path binary32 ops of IntersectsSphere
OPS_PER_PLANE_TEST = 17        # ... of IntersectPlane


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU).  Without a torch.distributed launcher (no WORLD_SIZE) and "
                         "N > 1, bench.py starts the N ranks itself (torch.distributed.run); every rank checks "
                         "WORLD_SIZE == N")
    ap.add_argument("--steps", type=int, default=1024, help="timed frames")
    ap.add_argument("--warmup", type=int, default=256, help="untimed frames first")
    ap.add_argument("--min-warmup-ms", type=float, default=50.0,
                    help="N=1: keep warming up (untimed, whole launches) until this much wall time has passed -- "
                         "the GPU needs ~10-50 ms of load to reach its steady clock; reported as warmup_effective")
    ap.add_argument("--config", default="C3",
                    help="the bench line's config (default C3: BASELINE configs[2], the north-star's 1080p depth-4 "
                         "target; C2 = configs[1] runs under 'also')")
    ap.add_argument("--also-dist", default="C5",
                    help="N>1: comma list of further configs run through the same band pipeline after --config and "
                         "reported under 'also' (default C5: 7680x4320, the config BASELINE names for the 1/2/4/8-GPU "
                         "scaling curve); '' = none")
    ap.add_argument("--also", default="C2,C4,C5",
                    help="N=1: comma list of further configs measured in the same run and reported under 'also' "
                         "(default C2, BASELINE configs[1]: depth 1, 1 light; C4, 3840x2160 with 64 spheres, "
                         "4 lights, depth 6 -- BASELINE's LDS/compaction stress config; and C5, the 7680x4320 "
                         "config of BASELINE's 1/2/4/8-GPU curve -- the N > 1 lines carry it as also.C5); '' = none")
    ap.add_argument("--tick-configs", default="C2,C4,C5",
                    help="configs whose plugin-path Tick() rates (rt_render / rt_render_async into registered host "
                         "memory, PCIe included) are reported under tick_by_config beside the bench config's own "
                         "(N > 1: rank 0's single-process Context(N) leg, plugin_tick); '' = none")
    ap.add_argument("--size", default="",
                    help="WxH: probe runs only -- the config's scene at another frame size (never the bench line)")
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--frames-per-launch", type=int, default=64,
                    help="N=1: at most this many frames per launch (rt_render_bands_batch: every frame traced in "
                         "full, the same camera); the steps are split into balanced launches (20 -> one of 20, "
                         "100 -> 50 + 50).  N>1 tiles: = --batch")
    ap.add_argument("--inflight", type=int, default=1,
                    help="launches in flight (a swap chain: one stream and one output buffer per slot).  1 (default): "
                         "the launches run alone, back to back, so kernel time x launches <= wall time")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N>1: gather each frame before tracing the next (no double buffering)")
    ap.add_argument("--batch", type=int, default=0,
                    help="N>1: frames per RCCL gather (pipelined; 1 = one gather per frame).  0 = auto: 64, "
                         "or the whole run when it is <= 128 frames (one batch).  A batch boundary costs the host "
                         "~100-200 us (codec calls, two collectives, a size read-back): at 16 frames per "
                         "gather that, not the GPU, bounded a rank's 1/8 share of 1080p (8.9 vs 3.0 us per "
                         "frame, tools/overhead_probe.sh)")
    ap.add_argument("--band-format", choices=["tiles", "rgb24", "int32"], default="tiles",
                    help="N>1: band sets shipped to rank 0 tile-encoded (lossless, rt_encode_bands), as packed "
                         "24-bit RGB or as int32 pixels")
    ap.add_argument("--rank0-codec", action="store_true",
                    help="N>1 tiles: rank 0 encodes and decodes its own bands too (instead of rendering them "
                         "straight into its frames); the one-process rehearsal uses it to exercise the codec")
    ap.add_argument("--no-fuse", action="store_true",
                    help="N>1 tiles: trace into an int32 band set and encode it (rt_encode_bands) instead of "
                         "tracing straight into the wire (rt_render_bands_tiles + rt_finish_wire: the encoder fused "
                         "into the trace kernel's epilogue, the band set never written)")
    ap.add_argument("--no-speculate", action="store_true",
                    help="N>1 tiles: read every batch's reduced wire size back before its gather (default: after "
                         "the warm-up, gather at 1.25 x the largest wire per frame seen so far right behind the size "
                         "reduce, check the reduced size before decoding and gather again when it was exceeded)")
    ap.add_argument("--spec-margin", type=float, default=1.25,
                    help="N>1 tiles: speculative gather size = this x the warm-up's largest wire per frame (< 1: "
                         "probe/test of the too-short path, which repeats a one-batch timed region)")
    ap.add_argument("--compositor", choices=["auto", "on", "off"], default="auto",
                    help="N>1 tiles: rank 0 traces nothing and assembles the frames that ranks 1..N-1 "
                         "trace as a band world of N-1 (auto: N >= 8, where rank 0's own share plus the "
                         "decode of the others' made it the slowest rank)")
    ap.add_argument("--rank0-share", default="auto",
                    help="N>1 tiles: rank 0's share of the frame -- auto: measured per leg (rank0_tail_rows: rank 0 "
                         "renders the frame's last rows itself, sized so that its trace plus the decode of the others' "
                         "bands take as long as their trace; 0 rows = the compositor, a share of 1/N or more = rank 0 "
                         "as an ordinary band rank); off: --compositor decides; an integer: that many last rows")
    ap.add_argument("--torch-collectives", action="store_true",
                    help="N>1 tiles: the size reduce and the gather through torch.distributed (its own collective "
                         "stream, waited on side streams) also for a run of one batch, instead of the library's RCCL "
                         "communicator on the trace/encode/decode stream (rt_comm_*)")
    ap.add_argument("--dist-path", action="store_true",
                    help="rehearsal: run the N>1 band/gather path even with one process (RCCL world of 1)")
    ap.add_argument("--no-verify", dest="verify", action="store_false",
                    help="N>1 path: skip the check after the timed run (default: rank 0 compares every frame still "
                         "in its frame rings -- tiles: all frames of a run of <= 3 batches -- with a single-launch "
                         "render of the same view, reports verified_frames, and every rank exits 3 on a mismatch)")
    ap.add_argument("--verify", dest="verify", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--master-port", type=int, default=29531, help="self-launch (--gpus N > 1): rendezvous port")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="rehearsal of the N > 1 path on fewer GPUs than ranks: the N ranks share the visible GPUs "
                         "(rank r on device r %% count) and the collectives run over gloo (RCCL refuses two ranks on "
                         "one GPU).  Exercises every rank's code path (bands, codec, pipelined gathers, compositor, "
                         "barrier and max-over-ranks timing); the line is marked 'rehearsal' and is not a result")
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="CPU baseline budget: 40 %% on the bench config, the rest on C3, C1 and the verbatim "
                         "reference scene")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-tick", action="store_true",
                    help="skip the Tick()-path probe and the work count (profiling runs: every trace dispatch of "
                         "the run then has the bench's launch shape)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="rocprofv3 PMC summary (HBM bytes per trace launch) for roofline.traffic")
    return ap.parse_args(argv)


def launch_command(argv, n, port):
    """The torch.distributed.run command line that starts n ranks of this script with argv."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def world_check(args, env=os.environ):
    """(action, message): 'run' in this process, 'spawn' the ranks, or 'fail'.

    Under a launcher every rank must see WORLD_SIZE == --gpus; without one, --gpus N > 1 spawns N
    ranks (the parent touches no GPU: it only counts devices, which does not initialise HIP)."""
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != args.gpus:
            return "fail", f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}"
        return "run", ""
    if args.gpus <= 1:
        return "run", ""
    return "spawn", ""


def device_count():
    import torch
    return torch.cuda.device_count()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cgroup_cpus():
    """CPU quota of this process's cgroup (cgroup v2 cpu.max), or None when unlimited/unknown."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if quota == "max" else float(quota) / float(period)
    except (OSError, ValueError):
        pass
    try:  # cgroup v1
        quota = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if quota <= 0 else quota / period
    except (OSError, ValueError):
        return None


def cgroup_throttle():
    """(nr_periods, nr_throttled, throttled_usec) of this cgroup's CPU controller (v2 cpu.stat, or v1
    cpu/cpu.stat with throttled_time in ns), or None when neither is readable."""
    for path, scale in (("/sys/fs/cgroup/cpu.stat", 1.0), ("/sys/fs/cgroup/cpu/cpu.stat", 1e-3)):
        try:
            kv = dict(line.split()[:2] for line in open(path) if len(line.split()) >= 2)
        except OSError:
            continue
        usec = kv.get("throttled_usec")
        usec = float(usec) if usec is not None else float(kv.get("throttled_time", 0)) * scale
        return int(kv.get("nr_periods", 0)), int(kv.get("nr_throttled", 0)), usec
    return None


def percentiles(xs, ps=(10, 50, 90)):
    """Nearest-rank percentiles of xs (sorted copy)."""
    s = sorted(xs)
    return [s[min(len(s) - 1, max(0, int(round(p / 100.0 * (len(s) - 1)))))] for p in ps]


def cpu_baseline(samples, seconds):
    """Reference-faithful CPU restatement (oracle, all-hit driver, column-outer/row-parallel loop
    like RayTracer.cs:898-901), timed on every core this process may run on, on whole frames.

    samples: [(scene, rays_per_frame, share of `seconds`)].  The first is the bench workload
    (the cpu_baseline value); the others are reported beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    # every CPU this process may use: its affinity set, capped by its cgroup's CPU quota (a GPU box
    # grants a 16-CPU share of a larger machine: more threads than the quota only get throttled)
    threads = max(1, min(affinity, int(quota + 0.5))) if quota else affinity
    out = None
    for scene, rays_per_frame, share in samples:
        if rays_per_frame is None:  # count the visible-path rays with the oracle's nearest driver
            _, ost = pyoracle.render(scene, pyoracle.MODE_NEAREST, threads)
            rays_per_frame = ost["primary_rays"] + ost["reflect_rays"] + ost["shadow_rays"]
        pyoracle.render(scene.resized(scene.width, 8), pyoracle.MODE_REFERENCE, threads)  # warm-up
        times = []
        thr0, cpu0, t_start = cgroup_throttle(), os.times(), time.perf_counter()
        while True:
            t0 = time.perf_counter()
            pyoracle.render(scene, pyoracle.MODE_REFERENCE, threads)
            times.append(time.perf_counter() - t0)
            if (time.perf_counter() - t_start > seconds * share and len(times) >= 3) or len(times) >= 200:
                break
        wall = time.perf_counter() - t_start
        thr1, cpu1 = cgroup_throttle(), os.times()
        p10, med, p90 = percentiles(times)
        entry = {"value": rays_per_frame / med / 1e6, "unit": "Mray/s", "fps": 1.0 / med, "frames": len(times),
                 "workload": f"{scene.name}: {scene.width}x{scene.height}, {len(scene.spheres)} spheres, "
                             f"{len(scene.lights)} lights, depth {scene.recursion_limit + 1}",
                 "frame_ms_p10_p50_p90": [round(x * 1e3, 3) for x in (p10, med, p90)],
                 # CPU time the process got per wall second: ~threads when every worker ran all the time
                 "cpus_scheduled": round(((cpu1.user - cpu0.user) + (cpu1.system - cpu0.system)) / wall, 2),
                 "cgroup_throttled": None if not (thr0 and thr1) else {
                     "periods": thr1[0] - thr0[0], "nr_throttled": thr1[1] - thr0[1],
                     "throttled_ms": round((thr1[2] - thr0[2]) / 1e3, 1)}}
        if out is None:
            out = dict(entry)
            out.update({
                "cores": threads, "kind": "port", "affinity_cpus": affinity, "nproc": os.cpu_count(),
                "cgroup_cpu_quota": quota,
                "sample": f"{len(times)} full {scene.width}x{scene.height} frames of {scene.name} (median), C "
                          f"restatement of RayTracer.cs (all-hit shading, per-pixel camera trig, column-outer/"
                          f"row-parallel loop), {threads} threads = every CPU this process may use "
                          f"(sched_getaffinity {affinity} CPUs, cgroup quota {quota if quota else 'none'} CPUs, "
                          f"os.cpu_count {os.cpu_count()}) on {cpu_model()}; the spread: frame_ms_p10_p50_p90, "
                          f"cpus_scheduled (process CPU time / wall) and the cgroup's throttling over the sample",
                "others": {},
            })
        else:
            out["others"][scene.name] = entry
    return out


def load_pmc(path, config, world):
    """PMC summary of the trace kernel for this config (tools/pmc_summary.py --json), or None."""
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(config, {}).get(str(world))
    except (OSError, ValueError):
        return None


def plan_launches(n, fpl):
    """Balanced launch sizes for n frames, at most fpl per launch (20 -> [20], 100 -> [50, 50])."""
    if n <= 0:
        return []
    k = -(-n // fpl)
    base, extra = divmod(n, k)
    return [base + 1] * extra + [base] * (k - extra)


def measure_single(ctx, sc, args, torch, abi, steps, warmup):
    """N = 1: `steps` frames of `sc` in balanced launches of <= --frames-per-launch frames
    (rt_render_bands_batch: one launch, grid z = frame, every frame traced in full into its own
    slot), --inflight launches in flight.  Timed between two torch.cuda.synchronize() calls."""
    W, H = sc.width, sc.height
    nf = max(1, args.inflight)
    fpl = max(1, min(args.frames_per_launch, 65535))
    cap = max(plan_launches(steps, fpl) + plan_launches(max(1, warmup), fpl))
    bufs = [torch.empty(cap * W * H, dtype=torch.int32, device="cuda") for _ in range(nf)]
    stream = torch.cuda.current_stream()
    streams = [stream] + [torch.cuda.Stream() for _ in range(nf - 1)]
    k = [0]

    def issue(n, lim=fpl):
        for m in plan_launches(n, min(lim, cap)):
            if not 1 <= m <= cap:  # every launch must fit its output slot
                raise RuntimeError(f"launch of {m} frames exceeds the {cap}-frame buffer")
            i = k[0] % nf
            k[0] += 1
            ctx.render_bands_batch(W, H, H, 0, 1, m, bufs[i].data_ptr(), W * H * 4, abi.RT_BANDS_INT32,
                                   streams[i].cuda_stream)

    # One launch in flight: no event pairs inside the timed region (each pair around a launch costs
    # ~9 us of GPU time, tools/region_probe.py); the events around the region measure the launches,
    # and an untimed pass of the same launches afterwards brackets each one (cross-check).
    # Overlapping launches (--inflight > 1): a sampled pair per 4 launches.
    ctx.set_timing(0 if nf == 1 else 4)
    t_w = time.perf_counter()
    issue(warmup)
    torch.cuda.synchronize()
    done = warmup
    while (time.perf_counter() - t_w) * 1e3 < args.min_warmup_ms:  # clock ramp (untimed)
        per_frame = (time.perf_counter() - t_w) / max(1, done)
        n = max(1, min(16 * fpl, int((args.min_warmup_ms / 1e3 - (time.perf_counter() - t_w)) / per_frame) + 1))
        n = -(-n // cap) * cap  # whole launches of `cap` frames: every warm-up launch has the timed shape
        issue(n)
        done += n
        torch.cuda.synchronize()
    ctx.reset_stats()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)  # the first record of an event creates it (~10 us of host time): not in the region
    ev1.record(stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)  # on the launch stream(s): the others start after it, it ends after them
    for s in streams[1:]:
        s.wait_event(ev0)
    issue(steps)
    host_s = (time.perf_counter() - t0) / max(1, steps)  # host issue time per step
    for s in streams[1:]:
        stream.wait_stream(s)
    ev1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    launch_s = None
    if nf == 1:  # cross-check (untimed): the same launches, an event pair around each
        ctx.set_timing(1)
        ctx.reset_stats()
        issue(steps)
        torch.cuda.synchronize()
        s2 = ctx.stats()
        launch_s = s2["kernel_ms"] / 1e3 / s2["timed_launches"] if s2["timed_launches"] else None
    ctx.set_timing(64)  # the library's default sampling
    return {"elapsed": elapsed, "period_s": ev0.elapsed_time(ev1) / 1e3 / steps, "stats": st, "host_s": host_s,
            "launches": len(plan_launches(steps, fpl)), "warmup_effective": done, "inflight": nf,
            "launch_events_s": launch_s}


def single_summary(sc, m, steps):
    """Per-config numbers of an N = 1 measurement (value, roofline inputs)."""
    st = m["stats"]
    rays = st["primary_rays"] + st["reflect_rays"] + st["shadow_rays"]
    W, H = sc.width, sc.height
    launches = m["launches"]
    frames_per_launch = steps / launches
    if m["inflight"] == 1:  # launches back to back on one stream: the region's events / launches
        kernel_s = m["period_s"] * steps / launches
    else:  # overlapping launches: the sampled per-launch event pairs
        kernel_s = st["kernel_ms"] / 1e3 / max(1, st["timed_launches"]) if st["timed_launches"] else m["period_s"]
    achieved = 4.0 * W * H * frames_per_launch / kernel_s / 1e9
    return {
        "value": rays / m["elapsed"] / 1e6, "unit": "Mray/s", "ms_per_step": m["elapsed"] * 1e3 / steps,
        "fps": steps / m["elapsed"], "rays_per_frame": rays / steps,
        "workload": f"{sc.name}: {sc.note}", "kernel": "trace_direct_kernel" if len(sc.spheres) < 12
        else "trace_bundle_kernel",
        "kernel_avg_ms": kernel_s * 1e3, "kernel_ms_per_frame": kernel_s * 1e3 / frames_per_launch,
        "frames_per_launch": frames_per_launch, "launches": launches, "timed_launches": st["timed_launches"],
        "kernel_avg_ms_launch_events": m["launch_events_s"] * 1e3 if m["launch_events_s"] else None,
        "frame_period_ms": m["period_s"] * 1e3, "hbm_gbs": achieved, "hbm_frac": achieved / HBM_PEAK_GBS,
        "f_alg": OPS_PER_SPHERE_TEST * st["sphere_tests"] + OPS_PER_PLANE_TEST * st["plane_tests"],
    }


def tick_rates(ctx, W, H, torch, n=20, reps=3, n_single=200):
    """The interactive shapes beside the batched headline (never `value`); each the median of
    `reps` runs of n frames, same camera:
    - single_launch_fps: rt_render_device, one frame per launch, device-resident (what a Tick()
      loop issues, without the PCIe hand-off), over runs of n_single frames: a display loop's
      steady rate (single_launch_fps_20: runs of 20, where the first launch's start and the closing
      synchronisation, ~50 us together, are spread over 20 frames only);
    - tick_fps_incl_d2h: rt_render, the synchronous Tick() (trace + D2H into the caller's
      registered buffer, returns with the frame complete);
    - tick_async_fps_incl_d2h: rt_render_async into two alternating registered buffers and an
      rt_wait per pair (a display loop two frames deep);
    - tick_async_deep_fps_incl_d2h: n frames queued into n registered buffers, one rt_wait.
    rt_render_async's D2H of frame k rides in frame k+1's launch (copy slice) or rt_wait's.
    Every shape runs with the work counters off (rt_set_counting(0), what the plugin's display loop sets:
    the reference's Tick counts nothing); they are on again on return."""
    import numpy as np
    ctx.set_counting(False)

    def med(fn, frames=n):
        fn()  # warm
        rates = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            rates.append(frames / (time.perf_counter() - t))
        return sorted(rates)[len(rates) // 2], [round(r, 1) for r in rates]

    dev = torch.empty(W * H, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()

    def single_of(frames):
        def run():
            for _ in range(frames):
                ctx.render_device(W, H, dev.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
        return run
    hosts = [np.zeros(W * H, dtype=np.int32) for _ in range(n)]
    for hb in hosts:
        ctx.register_host(hb)

    def sync():
        for _ in range(n):
            ctx.render(W, H, hosts[0])

    def pair():
        for k in range(n):
            ctx.render_async(W, H, hosts[k % 2])
            if k % 2:
                ctx.wait()
        ctx.wait()

    def deep():
        for k in range(n):
            ctx.render_async(W, H, hosts[k])
        ctx.wait()
    out = {}
    out["single_launch_fps"], out["single_launch_fps_runs"] = med(single_of(n_single), n_single)
    for key, fn in (("single_launch_fps_20", single_of(n)), ("tick_fps_incl_d2h", sync),
                    ("tick_async_fps_incl_d2h", pair), ("tick_async_deep_fps_incl_d2h", deep)):
        out[key], out[key + "_runs"] = med(fn)
    for hb in hosts:
        ctx.unregister_host(hb)
    ctx.set_counting(True)
    out["tick_note"] = (f"median of {reps} runs each; single_launch_fps = rt_render_device one frame per launch into "
                        f"HBM, runs of {n_single} frames (single_launch_fps_20: runs of {n}); tick_* runs of {n} "
                        f"frames, including the D2H into registered host memory (PCIe); work counters off "
                        f"(rt_set_counting(0), the display loop's setting)")
    return out


def lone_frame_rate(ctx, W, H, torch, frames, reps=3, warm=48):
    """One frame per launch (rt_render_device into HBM, the display loop's shape; never `value`) for an `also`
    config, counters off: `warm` launches first (the library's dispatch-order tuner measures its candidates and
    keeps one), then the median of `reps` runs of `frames` launches."""
    ctx.set_counting(False)
    dev = torch.empty(W * H, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run(k):
        for _ in range(k):
            ctx.render_device(W, H, dev.data_ptr(), st)
        torch.cuda.synchronize()
    for _ in range(warm // 8):
        run(8)
    rates = []
    for _ in range(reps):
        t = time.perf_counter()
        run(frames)
        rates.append(frames / (time.perf_counter() - t))
    ctx.set_counting(True)
    fps = sorted(rates)[len(rates) // 2]
    return {"single_launch_fps": fps, "single_launch_ms": 1e3 / fps, "single_launch_fps_runs": [round(r, 1) for r in rates],
            "dispatch_order": ctx.dispatch_order()}


def plugin_ticks(ctx, configs, scenes, n=20, reps=3):
    """The plugin path's Tick() per config (RayTracer.Tick -> rt_render / rt_render_async into registered
    host buffers, the frame complete in host memory -- PCIe included; never `value`), median of `reps` runs
    of n frames: tick_fps (synchronous), tick_async_fps (two frames deep, a wait per pair) and the frame
    bytes per second they move to the host (d2h_gbs).  ctx: a Context of any worker count (its devices
    each hand their own bands over their own link)."""
    import numpy as np
    out = {}
    ctx.set_counting(False)  # the display loop's setting (the plugin shim's), as tick_rates
    for name in configs:
        sc = scenes.config(name)
        W, H = sc.width, sc.height
        ctx.set_scene(sc)
        bufs = [np.zeros(W * H, dtype=np.int32) for _ in range(2)]
        for b in bufs:
            ctx.register_host(b)

        def sync():
            for _ in range(n):
                ctx.render(W, H, bufs[0])

        def pair():
            for k in range(n):
                ctx.render_async(W, H, bufs[k % 2])
                if k % 2:
                    ctx.wait()
            ctx.wait()
        e = {}
        for key, fn in (("tick_fps", sync), ("tick_async_fps", pair)):
            fn()  # warm
            rates = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                rates.append(n / (time.perf_counter() - t))
            e[key] = sorted(rates)[len(rates) // 2]
            e[key + "_runs"] = [round(r, 1) for r in rates]
            e[key.replace("fps", "d2h_gbs")] = W * H * 4 * e[key] / 1e9
        e["frame_mb"] = W * H * 4 / 1e6
        for b in bufs:
            ctx.unregister_host(b)
        out[sc.name] = e
    ctx.set_counting(True)
    return out


def main():
    args = parse()
    action, msg = world_check(args)
    if action == "fail":
        print(msg, file=sys.stderr, flush=True)
        sys.exit(2)
    if action == "spawn":
        n = device_count()
        if n < args.gpus and not (args.rehearse_gloo and n >= 1):
            print(f"bench.py --gpus {args.gpus}: only {n} GPU(s) visible", file=sys.stderr, flush=True)
            sys.exit(2)
        sys.exit(subprocess.call(launch_command(sys.argv[1:], args.gpus, args.master_port)))
    args.auto_batch = args.batch <= 0
    if args.batch <= 0:
        # N > 1: a short run is one batch (one size reduce + one gather + one decode: the fixed
        # latency of each collective and of the host's size read-back dominates a handful of
        # 1080p frames, and a pipeline of small batches pays it per batch); long runs pipeline
        # batches of 64 frames.  The tile pipeline refines this per leg (auto_batch_frames).
        args.batch = args.steps if args.steps <= 128 else 64
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    from raytracer_hip import Context, abi, scenes
    if not os.path.exists(abi.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)

    if world == 1 and not args.dist_path:
        return main_single(args, torch, Context, abi, scenes)

    # N > 1 (or the one-process rehearsal of that path): one process per GPU, RCCL process group
    # (--rehearse-gloo: the ranks share the visible GPUs and talk over gloo)
    if args.rehearse_gloo:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    if args.rehearse_gloo:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    out = dist_leg(args, args.config, rank, world, local, torch, dist, Context, abi, scenes, size=args.size)
    # further configs through the same pipeline (default C5: 7680x4320, the configuration BASELINE
    # names for the 1/2/4/8-GPU scaling curve), each with its own value / ms_per_step / n_gpus
    also = [c for c in (x.strip() for x in args.also_dist.split(",")) if c and c.upper() != args.config.upper()]
    for name in also:
        o2 = dist_leg(args, name, rank, world, local, torch, dist, Context, abi, scenes)
        if rank == 0:
            out.setdefault("also", {})[o2["config"]["workload"].split(":")[0]] = {
                k: o2[k] for k in ("value", "unit", "n_gpus", "steps", "ms_per_step", "fps", "config", "roofline",
                                   "verified_frames") if k in o2}
    tick_cfgs = [c for c in (x.strip() for x in args.tick_configs.split(",")) if c]
    if not args.no_tick and (tick_cfgs or args.config) and world > 1:
        # The plugin path's own multi-GPU Tick() (what RayTracer.Tick with RT_GPUS = N runs): ONE process,
        # Context(N) -- every device traces its interleaved bands and hands them to the host frame over its
        # own PCIe link.  Rank 0 drives all N devices; the other ranks wait at a barrier on the host (a gloo
        # group: an RCCL barrier would leave a spinning collective kernel on each of their GPUs while rank 0's
        # workers trace there).  (The rehearsal on fewer GPUs: the N workers share the device,
        # RT_CREATE_SHARED_DEVICE.)
        torch.cuda.synchronize()
        host_pg = None
        if not args.rehearse_gloo:
            try:  # (every rank calls new_group; a failure falls back to the default group's barrier)
                host_pg = dist.new_group(backend="gloo")
            except Exception as e:  # noqa: BLE001
                print(f"plugin_tick: no gloo group ({e!r}); RCCL barrier instead", file=sys.stderr, flush=True)
        dist.barrier(group=host_pg)
        if rank == 0:
            try:
                flags = abi.RT_CREATE_SHARED_DEVICE if args.rehearse_gloo else 0
                with Context(world, flags) as pctx:
                    pt = plugin_ticks(pctx, [args.config] + [c for c in tick_cfgs if c != args.config], scenes)
                pt["n_workers"] = world
                pt["note"] = (f"single process, Context({world}){' shared-device rehearsal' if flags else ''}: "
                              f"rt_render (synchronous) / rt_render_async (two frames deep) into registered host "
                              f"buffers, every device's bands over its own PCIe link; median of 3 runs of 20 frames")
            except Exception as e:  # reported, never fatal for the line
                pt = {"error": repr(e)}
            out["plugin_tick"] = pt
        dist.barrier(group=host_pg)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def auto_batch_frames(ctx, W, H, rb, band_rank, band_world, idle, steps, torch, dist, target_s=1e-3, max_batches=4):
    """Frames per gather for a run of `steps` <= 128 frames (every rank takes part; all get the same
    answer).  One batch when the run's trace is short (C2: the fixed latency of each collective, the
    size read-back and the decode dominate, and one batch can use the library's collectives on the
    trace stream); otherwise up to `max_batches` batches of >= `target_s` of trace each, so that the
    gather and rank 0's decode of batch b run under the trace of batch b+1 instead of after the whole
    run (C5: a 1080p-sized wire per rank per frame is megabytes -- ~1 ms of gather and 0.7 ms of
    decode for 20 frames at N = 8, ~3.7 ms of gather over one link at N = 2).  The per-frame trace time
    of this rank's share comes from a 2-frame launch after a warm one, the max over ranks."""
    import time as _t
    t = 0.0
    if not idle and rb.slot_elems > 0:
        from raytracer_hip import abi as _abi
        buf = torch.empty(2 * rb.slot_elems, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = _t.perf_counter()
            ctx.render_bands_batch(W, H, rb.band_rows, band_rank, band_world, 2, buf.data_ptr(), rb.slot_elems * 4,
                                   _abi.RT_BANDS_INT32, st)
            torch.cuda.synchronize()
            t = (_t.perf_counter() - t0) / 2
        del buf
    tt = torch.tensor([t], dtype=torch.float64, device="cuda")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    k = max(1, min(max_batches, int(round(steps * float(tt) / target_s))))
    return -(-steps // k)


# Rank 0's decode of the other ranks' wires per pixel of the frame (rt_decode_gathered; profiles/r04_dist_stages.txt:
# 45.4 us for 20 C2 frames in one batch, 2.0-2.1 us per 1080p frame at 64 frames per batch)
DECODE_S_PER_PX = 1.1e-12


def solve_rank0_tail(T, D, H, band_rows, world, probe):
    """rank0_tail_rows' model: T = s per whole frame's trace, D = s per whole frame's decode, probe(rows) = s per
    frame of the last `rows` rows.  Solves t(h) + D (H - h) / H = (T - t(h)) / (N - 1) with t(h) ~ c h, c measured at
    the uniform share and then once more at the solution.  Returns (h in whole bands, the uniform share hu, c);
    h >= hu means rank 0 stays interleaved, 0 the compositor."""
    hu = max(band_rows, (H // world) // band_rows * band_rows)  # the uniform share, whole bands
    h, c = float(hu), probe(hu) / hu
    for _ in range(2):  # the linear model, then once more with the slope measured at its solution
        denom = c * world / (world - 1) - D / H
        h = (T / (world - 1) - D) / denom if denom > 0 else 0.0
        hb = int(h // band_rows) * band_rows
        if hb <= 0 or hb >= hu:
            break
        c = probe(hb) / hb
    return int(max(0.0, h) // band_rows) * band_rows, hu, c


def rank0_tail_rows(ctx, W, H, band_rows, world, rank, torch, dist, log=None):
    """Rank 0's share of an N > 1 leg (every rank takes part and gets the same answer): -1 = rank 0 is an
    ordinary band rank (interleaved 1/N), 0 = compositor (rank 0 only decodes), h > 0 = rank 0 renders
    the frame's last h rows (whole bands) itself and ranks 1..N-1 the rows above them.  Rank 0 measures
    the full frame's trace T and the trace of a candidate tail t(h) (4-frame launches, HIP events, best of 3
    after a warm one, every rank idle)
    and solves  t(h) + D (H - h) / H = (T - t(h)) / (N - 1)  for h with t(h) ~ c h (c from the probe,
    refined once at the solution), D = the decode of a whole frame (DECODE_S_PER_PX).  A
    solution at or above the uniform share 1/N keeps rank 0 interleaved."""
    from raytracer_hip import abi as _abi
    ans = torch.tensor([-1.0], dtype=torch.float64, device="cuda")
    # every rank idle first: on a shared-GPU rehearsal another rank's set-up work would land in rank 0's probe
    torch.cuda.synchronize()
    dist.barrier() if world > 1 else None
    if rank == 0:
        frames = 4
        buf = torch.empty(frames * W * H, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def probe(rows):  # s per frame of the last `rows` rows (rows = H: the whole frame): best of 3 after a warm one
            best = float("inf")
            for k in range(4):
                e0.record(st)
                ctx.render_bands_batch(W, H, band_rows, (H - rows) // band_rows, 1, frames, buf.data_ptr(), W * H * 4,
                                       _abi.RT_BANDS_FRAME, st.cuda_stream)
                e1.record(st)
                e1.synchronize()
                if k:
                    best = min(best, e0.elapsed_time(e1) * 1e-3 / frames)
            return best
        T = probe(H)
        D = DECODE_S_PER_PX * W * H
        hb, hu, c = solve_rank0_tail(T, D, H, band_rows, world, probe)
        ans[0] = -1.0 if hb >= hu else float(hb)
        if log:
            log(f"rank 0 share: T {T * 1e6:.1f} us/frame, decode {D * 1e6:.1f} us/frame, tail slope "
                f"{c * 1e9:.1f} ns/row, uniform {hu} rows -> {'interleaved' if hb >= hu else f'{hb} tail rows'}")
        del buf
    dist.all_reduce(ans, op=dist.ReduceOp.MAX) if world > 1 else None
    return int(ans.item())


def dist_leg(args, config_name, rank, world, local, torch, dist, Context, abi, scenes, size=""):
    """One N > 1 measurement of `config_name` through the band pipeline (rank 0 returns the
    line's dict, the other ranks None).  Every rank runs every leg, so the collectives match."""
    sc = scenes.config(config_name)
    if size:  # probe runs only (--size): the config's scene at another frame size
        w_, h_ = map(int, size.lower().split("x"))
        sc = sc.resized(w_, h_, f"{sc.name}@{w_}x{h_}")
    W, H = sc.width, sc.height
    ctx = Context(1)
    ctx.set_scene(sc)
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream

    def finish():
        pass

    streams = [stream]
    tg = None  # tile-encoded gather (--band-format tiles)
    run = None  # run(n): n steps (frames); else one step() per frame
    distributed = True
    comp = False  # compositor geometry (ranks 1..N-1 trace the frame, or all of it above rank 0's tail)
    tail = 0      # rank 0's last rows (with comp): it renders them itself
    Hc = H        # the band geometry's rows (H - tail)
    if True:
        from raytracer_hip.dist import BandGather, BatchedBandGather, RowBands
        tiles_ok = args.band_format == "tiles" and not args.no_pipeline and not args.rank0_codec and world >= 2
        share = -1
        if tiles_ok and args.rank0_share != "off":
            share = (rank0_tail_rows(ctx, W, H, args.band_rows, world, rank, torch, dist,
                                     lambda m: print(f"[{sc.name}] {m}", file=sys.stderr, flush=True))
                     if args.rank0_share == "auto" else int(args.rank0_share))
            comp = share >= 0
            tail = max(0, share)
        elif tiles_ok:
            comp = args.compositor == "on" or (args.compositor == "auto" and world >= 8)
        Hc = H - tail
        # band geometry: the process group's, or (compositor) ranks 1..N-1 as band ranks 0..N-2 of the
        # frame's first Hc rows, traced with the whole frame's view
        band_rank, band_world = (max(0, rank - 1), world - 1) if comp else (rank, world)
        if tail and rank > 0:
            ctx.set_view_height(H)
        rb = RowBands(W, Hc, args.band_rows, band_rank, band_world)
        launch_frames = 1
        px_per_launch = rb.pixels
        frame = torch.empty(W * H, dtype=torch.int32, device="cuda") if rank == 0 else None

        def scatter(parts):
            if rank == 0 and parts is not None:
                for r in range(world):
                    ctx.scatter_bands(W, H, rb.band_rows, r, world, parts[r].data_ptr(), frame.data_ptr(), s)

        if args.no_pipeline:
            if args.band_format == "tiles":
                raise SystemExit("--no-pipeline ships raw band sets: use --band-format int32/rgb24")
            bg = BandGather(rb, torch.device("cuda", local))

            def step():
                # trace this rank's bands -> RCCL gather of the slots to rank 0 -> reassemble there
                ctx.render_bands(W, H, rb.band_rows, rank, world, bg.local.data_ptr(), s)
                scatter(bg.gather())
        elif args.band_format == "tiles":
            from raytracer_hip import wire_layout
            from raytracer_hip.dist import TileBandGather

            def t_encode(raw, n, wire, size, st):
                if raw is None:  # fused: the batch was traced into the wire; finish it
                    ctx.finish_wire(W, Hc, rb.band_rows, band_rank, band_world, n, wire.data_ptr(), size.data_ptr(),
                                    st.cuda_stream)
                else:
                    ctx.encode_bands(W, Hc, rb.band_rows, band_rank, band_world, raw.data_ptr(), rb.slot_elems, n,
                                     wire.data_ptr(), size.data_ptr(), st.cuda_stream)

            def t_decode(recv, rank_stride, n, frames_, st, first_rank):
                # (rows [0, Hc) of each W x H frame: the band geometry's; rank 0 renders any rows below)
                ctx.decode_gathered(W, Hc, rb.band_rows, band_world, recv.data_ptr(), rank_stride, n,
                                    frames_.data_ptr(), W * H, st.cuda_stream, first_rank=first_rank)

            batch = args.batch
            if args.auto_batch and args.steps <= 128:
                batch = auto_batch_frames(ctx, W, Hc, rb, band_rank, band_world, comp and rank == 0, args.steps,
                                          torch, dist)
            coll = None
            if not args.rehearse_gloo and not args.torch_collectives and batch >= args.steps:
                # a run of one batch (the driver's --steps 20; each warm-up batch is drained too): the size
                # reduce and the gather through the library's RCCL communicator on the stream that traces,
                # encodes and decodes -- no hops into and out of torch.distributed's collective stream
                # (~20 us each, profiles/r03_dist_stages.txt).  Pipelined runs keep torch.distributed on
                # side streams, where the gather of batch b-1 overlaps the trace of batch b.
                from raytracer_hip.dist import LibraryCollectives

                def agree_min(v):
                    t = torch.tensor([v], dtype=torch.int32, device="cuda")
                    dist.all_reduce(t, op=dist.ReduceOp.MIN)
                    return int(t.item())
                try:  # (collective; every decision inside is taken alike on every rank)
                    coll = LibraryCollectives(ctx, rank, world, lambda t: dist.broadcast(t, src=0), agree_min)
                except Exception as e:  # CommUnavailable on every rank, or rt_comm_init failed on this one
                    print(f"[rank {rank}] library communicator unavailable ({e}); torch.distributed collectives",
                          file=sys.stderr, flush=True)
                    coll = None
                if agree_min(1 if coll is not None else 0) == 0:  # one choice for every rank
                    coll = None
            tg = TileBandGather(rb, torch.device("cuda", local), batch,
                                lambda n: wire_layout(W, Hc, rb.band_rows, band_world, n), t_encode, t_decode,
                                rank0_codec=args.rank0_codec, compositor=comp, phys_rank=rank, phys_world=world,
                                fused=not args.no_fuse, coll=coll, main_stream=stream, tail_rows=tail)
            out_fmt = abi.RT_BANDS_FRAME if tg.direct else abi.RT_BANDS_INT32
            # frames alternate between trace streams (two in flight per rank); at a batch end the
            # encode runs on `stream` after the others joined it, and the trace streams then wait
            # for it (the next-but-one batch reuses the raw buffer); collectives are waited on
            # the gather's own side streams, never on a trace stream.  Rank 0 renders its own
            # bands straight into its frame ring (RT_BANDS_FRAME): they never cross xGMI
            tstreams = [stream] + [torch.cuda.Stream() for _ in range(max(1, args.inflight) - 1)]
            stride_b = (W * H if tg.direct else rb.slot_elems) * 4
            launch_frames = tg.F
            px_per_launch = tg.F * (tail * W if (tail and rank == 0) else rb.pixels)
            if rank == 0:
                frame = None  # the decoded frames live in tg.frames (rings of F)

            def run(n):  # noqa: F811
                # one launch per batch (F frames of this rank's bands, each in full; a rank's share
                # of a 1080p frame is too little GPU work for a launch per frame), batches
                # alternating between the trace streams; at a batch end the encode runs on
                # `stream` after the batch's stream joined it, and every trace stream waits for it
                # (the next-but-one batch reuses the raw buffer, on any of them at --inflight >= 3)
                done = 0
                while done < n:
                    m = min(tg.F - tg.k % tg.F, n - done)
                    ts = tstreams[(tg.k // tg.F) % len(tstreams)]
                    if tg.k % tg.F == 0:
                        tg.begin_batch([ts])
                    if tg.fused:  # straight into the batch's wire (tile headers + codec scratch)
                        ctx.render_bands_tiles(W, Hc, rb.band_rows, band_rank, band_world, tg.k % tg.F, m, tg.F,
                                               tg.wire_target().data_ptr(), ts.cuda_stream)
                    elif tail and rank == 0:  # rank 0's share: the frame's last `tail` rows, into its frames
                        ctx.render_bands_batch(W, H, rb.band_rows, Hc // rb.band_rows, 1, m, tg.target().data_ptr(),
                                               stride_b, abi.RT_BANDS_FRAME, ts.cuda_stream)
                    elif not tg.idle:  # (the compositor rank only assembles)
                        ctx.render_bands_batch(W, H, rb.band_rows, band_rank, band_world, m, tg.target().data_ptr(),
                                               stride_b, out_fmt, ts.cuda_stream)
                    end = (tg.k + m) % tg.F == 0
                    if end and ts is not stream:
                        stream.wait_stream(ts)
                    for _ in range(m):
                        tg.commit(stream)
                    if end:
                        for t in tstreams[1:]:
                            t.wait_stream(stream)
                    done += m

            def finish():  # noqa: F811  -- the last (possibly partial) batch, every stage
                for t in tstreams[1:]:
                    stream.wait_stream(t)
                tg.drain(stream)
                stream.wait_stream(tg.comm)
                stream.wait_stream(tg.dec)
                for t in tstreams[1:]:  # (the next run's batches reuse the raw buffers)
                    t.wait_stream(stream)
        else:
            fmt = abi.RT_BANDS_RGB24 if args.band_format == "rgb24" else abi.RT_BANDS_INT32
            bgb = BatchedBandGather(rb, torch.device("cuda", local), frames_per_batch=args.batch,
                                    bpp=3 if fmt == abi.RT_BANDS_RGB24 else 4)

            def reassemble(done):
                # rank 0: one launch per frame puts every rank's bands into the frame
                if rank == 0:
                    for buf, n in done:
                        for f in range(n):
                            ctx.scatter_gathered(W, H, rb.band_rows, world, buf.data_ptr() + f * bgb.slot_bytes,
                                                 bgb.rank_stride, frame.data_ptr(), fmt, s)

            # frames of a batch alternate between trace streams (two frames in flight per rank);
            # the batch's gather is issued on `stream` after it has joined the others, and every
            # trace stream waits for the previous gather (whose buffer the next batch reuses)
            tstreams = [stream] + [torch.cuda.Stream() for _ in range(max(1, args.inflight) - 1)]

            def join_traces():
                for t in tstreams[1:]:
                    stream.wait_stream(t)

            def after_gather_wait():
                for t in tstreams[1:]:
                    t.wait_stream(stream)

            def step():
                # trace frame k's bands into its slot of the current batch; every F frames one
                # gather ships the batch to rank 0 while the next batch is traced
                k = bgb.k
                ctx.render_bands_ex(W, H, rb.band_rows, rank, world, bgb.frame_buffer(), fmt,
                                    tstreams[k % len(tstreams)].cuda_stream)
                if (k + 1) % bgb.F == 0:
                    join_traces()
                done = bgb.commit()
                if (k + 1) % bgb.F == 0:
                    after_gather_wait()
                if done is not None:
                    reassemble([done])

            def finish():  # noqa: F811  -- the last (possibly partial) batch
                join_traces()
                reassemble(bgb.drain())

    if run is None:
        def run(n):  # noqa: F811
            for _ in range(n):
                step()

    # no event pairs around the launches of the timed region (each pair costs ~9 us of GPU time,
    # tools/region_probe.py): the kernel duration comes from an untimed second pass (below)
    ctx.set_timing(0)
    if tg is not None and not tg.idle and not tg.direct and not tg.fused:
        # size the codec's scratch for a whole batch before anything is timed (rt_encode_bands grows
        # it on demand, behind a device synchronisation)
        t_encode(tg.raw[0], tg.F, tg.wire[0], tg.size[0], stream)
        torch.cuda.synchronize()
    # warm-up: --warmup frames, then whole batches until every rank has run for --min-warmup-ms
    # (the clock ramp); the ranks agree on each extra batch through an all_reduce, so every rank
    # issues the same collectives
    run(args.warmup)
    finish()
    torch.cuda.synchronize()
    warmup_done = args.warmup
    t_w = time.perf_counter()
    while True:
        more = torch.tensor([1.0 if (time.perf_counter() - t_w) * 1e3 < args.min_warmup_ms else 0.0],
                            dtype=torch.float64, device="cuda")
        dist.all_reduce(more, op=dist.ReduceOp.MAX)
        if float(more) == 0.0:
            break
        run(launch_frames)
        finish()
        torch.cuda.synchronize()
        warmup_done += launch_frames
    if tg is not None and not args.no_speculate:
        tg.set_capacity(args.spec_margin)  # the warm-up's largest wire per frame x 1.25 (checked per batch)

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)  # the first record of an event creates it (~10 us of host time): not in the region
    ev1.record(stream)
    # A run of one speculative batch on GPUs checks its reduced wire size after the region's closing
    # synchronisation instead of behind a host wait in its middle (TileBandGather.defer_checks); if the
    # size outgrew the speculative gather (every rank sees the same reduced size), the frames are not
    # final and the whole timed region is run again without speculation -- that run is reported.
    defer = (tg is not None and tg.cuda and tg.capacity_per_frame is not None and tg.F >= args.steps
             and not args.rehearse_gloo and not os.environ.get("RT_BENCH_NO_DEFER"))

    def region():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)  # on the launch stream(s): the others start after it, it ends after them
        for st_ in streams[1:]:
            st_.wait_event(ev0)
        run(args.steps)
        host_s = (time.perf_counter() - t0) / max(1, args.steps)  # host issue time per step (incl. any waits)
        finish()
        for st_ in streams[1:]:
            stream.wait_stream(st_)
        ev1.record(stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, host_s  # this rank's time; the line reports the max over ranks

    (elapsed, host_s), repeats = timed_attempts(ctx, tg, defer, region, dist.barrier if distributed else None,
                                                 lambda m: print(f"[rank {rank}] {m}", file=sys.stderr, flush=True))

    st = ctx.stats()
    rays = st["primary_rays"] + st["reflect_rays"] + st["shadow_rays"]
    f_alg = OPS_PER_SPHERE_TEST * st["sphere_tests"] + OPS_PER_PLANE_TEST * st["plane_tests"]
    period_s = ev0.elapsed_time(ev1) / 1e3 / args.steps
    # what the JSON line reports of the timed run, read before the second pass below
    gather_info = None
    if tg is not None:
        gather_info = {"bytes_sent": tg.bytes_sent, "speculative": tg.capacity_per_frame is not None,
                       "redone": tg.redone, "repeats": repeats}
    verified = None
    if args.verify:
        # rank 0 checks the decoded frames; every rank learns the outcome (and exits alike on a mismatch)
        verified, bad = verify_rings(ctx, tg, W, H, args.steps, torch) if rank == 0 else (0, 0)
        if distributed:
            flag = torch.tensor([bad], dtype=torch.int64, device="cuda")
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            bad = int(flag.item())
        if bad:
            print(f"[rank {rank}] verify: {sc.name} frames differ from a single-launch render", file=sys.stderr,
                  flush=True)
            sys.exit(3)
    # Kernel duration per launch: an untimed second pass of the same frames (same collectives on
    # every rank) with a HIP event pair around every launch on its own stream (rt_set_timing 1;
    # what rocprofv3's kernel trace reports too).  The frame period -- HIP events around the timed
    # region / steps -- is shorter when frames overlap.
    ctx.set_timing(1)
    ctx.reset_stats()
    run(args.steps)
    finish()
    torch.cuda.synchronize()
    st2 = ctx.stats()
    ctx.set_timing(64)  # the library's default sampling
    sampled_s = st2["kernel_ms"] / 1e3 / max(1, st2["timed_launches"])
    kernel_s = sampled_s if st2["timed_launches"] else period_s
    if distributed:
        t = torch.tensor([elapsed, float(rays), float(f_alg), kernel_s], dtype=torch.float64, device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, rays, kernel_s = float(tmax[0]), float(t[1]), float(tmax[3])
        f_alg = float(t[2])

    if rank == 0:
        steps = args.steps
        rays_per_frame = rays / steps
        achieved_gbs = 4.0 * px_per_launch / kernel_s / 1e9
        pmc = load_pmc(args.pmc, sc.name, world)
        # PMC summaries are per dispatch of `frames_per_launch` frames (tools/pmc.sh): per frame,
        # then per launch of this run
        pmc_frames = (pmc.get("frames_per_launch") or 1) if pmc else 1
        traffic = pmc["hbm_bytes_per_launch"] / pmc_frames * launch_frames if pmc else None
        valu_insts = (pmc.get("counters") or {}).get("SQ_INSTS_VALU") if pmc else None
        valu_frame = valu_insts / pmc_frames if valu_insts else None  # wave instructions per frame
        r0_note = ""
        if comp and tail:
            r0_note = (f" (rank 0 renders the last {tail} rows and decodes, ranks 1..N-1 trace the {Hc} above: "
                       f"measured share)")
        elif comp:
            r0_note = " (compositor: rank 0 decodes, ranks 1..N-1 trace)"
        brute_tops = (f_alg / steps / max(1, world - 1 if comp else world)) * launch_frames / kernel_s / 1e12
        out = {
            "metric": METRIC,
            "value": rays / elapsed / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "warmup_effective": warmup_done,
            "ms_per_step": elapsed * 1e3 / steps,
            "fps": steps / elapsed,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded SplitMix64 scene, BASELINE.json config; no assets needed)",
            "config": {
                "workload": f"{sc.name}: {sc.note}",
                "width": W, "height": H, "spheres": len(sc.spheres), "planes": len(sc.planes),
                "lights": len(sc.lights), "depth": sc.recursion_limit + 1,
                "parallelism": f"interleaved {args.band_rows}-row bands x {world - 1 if comp else world} ranks + RCCL gather to "
                "rank 0" + r0_note
                + (" [collectives: " + ("library RCCL on the trace stream" if (tg is not None and tg.coll is not None)
                                        else "torch.distributed") + "]")
                + (" (one gather per frame)" if args.no_pipeline else
                   f" ({tg.F if tg is not None else args.batch} frames per gather, {args.band_format} bands, double-buffered: the gather of "
                   f"one batch overlaps the trace of the next)"),
                "rays_per_frame": rays_per_frame,
                "rank0_tail_rows": tail if comp else None,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "trace_direct_kernel" if sc and len(sc.spheres) < 12 else "trace_bundle_kernel",
                "kernel_avg_ms": kernel_s * 1e3,
                "frames_per_launch": launch_frames,
                "kernel_avg_source": "an untimed second pass of the same run with a HIP event pair around every "
                                     "launch on its stream (rt_set_timing 1), max over ranks",
                "frame_period_ms": period_s * 1e3,
                "note": "algorithmic bytes = 4 B framebuffer store per pixel x pixels per launch; the path is "
                        "FP32-VALU-bound",
            },
            "roofline_valu": {
                "bound": "valu",
                # chip-level issue rate: SQ_INSTS_VALU (wave instructions per launch, PMC) x 64
                # lanes per frame, over the frame period (frames overlap when several are in flight)
                "achieved": valu_frame * 64 / period_s / 1e12 if valu_frame else None,
                "peak": VALU_PEAK_TOPS,
                "unit": "TOP/s",
                "frac": valu_frame * 64 / period_s / 1e12 / VALU_PEAK_TOPS if valu_frame else None,
                "achieved_per_launch": valu_frame * launch_frames * 64 / kernel_s / 1e12 if valu_frame else None,
                "brute_force_equiv": brute_tops,
                "brute_force_ops_per_launch": f_alg / steps / max(1, world - 1 if comp else world) * launch_frames,
                "note": "achieved = issued VALU lane-ops per frame (profiles/pmc_traffic.json SQ_INSTS_VALU x 64) / "
                        "frame period; achieved_per_launch uses the launch duration instead; brute_force_equiv = "
                        "24 ops per sphere test + 17 per plane test over every primitive (SURVEY.md 8d) / kernel "
                        "time -- above peak where culling skips tests",
            },
            "cpu_baseline": None,
            # host time spent issuing the timed steps, per step (includes the host's waits inside
            # the loop, e.g. the N>1 pipeline's size handshake): ~ms_per_step when host-bound
            "host_ms_per_step": host_s * 1e3,
        }
        if args.rehearse_gloo:
            out["rehearsal"] = (f"gloo: {world} ranks sharing {torch.cuda.device_count()} GPU(s) -- a check of the N > 1 "
                                f"code path, not a measurement")
        if gather_info is not None:
            # wire bytes each rank shipped per frame (max over ranks, as gathered), vs the raw band set
            out["config"]["gather_wire_bytes_per_frame"] = gather_info["bytes_sent"] / steps
            out["config"]["gather_rgb24_bytes_per_frame"] = 3 * rb.slot_elems
            out["config"]["gather_speculative"] = gather_info["speculative"]
            out["config"]["gather_redone_batches"] = gather_info["redone"]
            out["config"]["timed_region_repeats"] = gather_info["repeats"]
        if args.verify:
            out["verified_frames"] = verified
    ctx.close()
    return out if rank == 0 else None


def timed_attempts(ctx, tg, defer, region, barrier=None, log=None):
    """The N > 1 timed region, `region()` -> its timing, between two barriers.  A run of one
    speculative batch (defer) checks its reduced wire size after the region's closing synchronisation
    (TileBandGather.defer_checks); when the size outgrew the speculative gather (every rank sees the
    same reduced size, so every rank decides alike) the frames are not final and the region is run
    again with exact sizes -- that attempt is the one reported.  The library's ray/test counters and
    the gather's byte/redo counters are reset before each attempt, so they describe the reported
    attempt alone.  Returns (region's timing, repeats)."""
    repeats = 0
    timing = None
    for attempt in range(2):
        ctx.reset_stats()
        if tg is not None:
            tg.bytes_sent = 0
            tg.redone = 0
            tg.defer_checks = defer and attempt == 0
            if attempt == 1:
                tg.capacity_per_frame = None  # exact sizes: a host wait per batch, always final
        if barrier is not None:
            barrier()
        timing = region()
        if barrier is not None:
            barrier()
        if tg is None or not tg.defer_checks or tg.check_deferred():
            break
        repeats += 1
        if log is not None:
            log("a speculative gather was too short: timed region repeated with exact sizes")
    if tg is not None:
        tg.defer_checks = False
    return timing, repeats


def verify_rings(ctx, tg, W, H, steps, torch):
    """Rank 0 of the tile pipeline: every decoded frame left in the frame rings (the last
    batches) must equal a single-launch render of the same view (all frames share the camera).
    Returns (frames verified, 1 if one differed else 0)."""
    if tg is None or tg.frames is None:
        return 0, 0
    want = torch.empty(W * H, dtype=torch.int32, device="cuda")
    ctx.render_device(W, H, want.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    n = 0
    first_timed = tg.batch - -(-steps // tg.F)  # batches of the timed run (the warm-up was drained before)
    for b in range(max(first_timed, tg.batch - 3), tg.batch):  # the rings of the last (up to) 3 batches
        ring = tg.ring_of(b).view(tg.F, W * H)
        frames_in_batch = tg.F if (b < tg.batch - 1 or steps % tg.F == 0) else steps % tg.F
        for f in range(frames_in_batch):
            if not torch.equal(ring[f], want):
                bad = int((ring[f] != want).sum())
                print(f"verify: batch {b} frame {f}: {bad} pixels differ", file=sys.stderr, flush=True)
                return n, 1
            n += 1
    return n, 0


def main_single(args, torch, Context, abi, scenes):
    """N = 1: the bench config (+ --also configs) on cuda:0; prints the JSON line."""
    torch.cuda.set_device(0)
    sc = scenes.config(args.config)
    if args.size:
        w_, h_ = map(int, args.size.lower().split("x"))
        sc = sc.resized(w_, h_, f"{sc.name}@{w_}x{h_}")
    W, H = sc.width, sc.height
    steps = args.steps
    ctx = Context(1)
    ctx.set_scene(sc)
    m = measure_single(ctx, sc, args, torch, abi, steps, args.warmup)
    r = single_summary(sc, m, steps)
    pmc = load_pmc(args.pmc, sc.name, 1)
    # PMC summaries are per dispatch of `frames_per_launch` frames (tools/pmc.sh): per frame here
    pmc_frames = (pmc.get("frames_per_launch") or 1) if pmc else 1
    traffic = pmc["hbm_bytes_per_launch"] / pmc_frames * r["frames_per_launch"] if pmc else None
    valu_insts = (pmc.get("counters") or {}).get("SQ_INSTS_VALU") if pmc else None
    valu_frame = valu_insts / pmc_frames if valu_insts else None  # wave instructions per frame
    kernel_frame_s = r["kernel_ms_per_frame"] / 1e3
    isolated = m["inflight"] == 1
    out = {
        "metric": METRIC,
        "value": r["value"],
        "unit": "Mray/s",
        "n_gpus": 1,
        "steps": steps,
        "warmup": args.warmup,
        "warmup_effective": m["warmup_effective"],
        "ms_per_step": r["ms_per_step"],
        "fps": r["fps"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded SplitMix64 scene, BASELINE.json config; no assets needed)",
        "config": {
            "workload": r["workload"],
            "width": W, "height": H, "spheres": len(sc.spheres), "planes": len(sc.planes),
            "lights": len(sc.lights), "depth": sc.recursion_limit + 1,
            "parallelism": f"single GPU, {r['launches']} balanced launches of <= {args.frames_per_launch} frames "
                           f"(rt_render_bands_batch), {m['inflight']} in flight",
            "rays_per_frame": r["rays_per_frame"],
        },
        "roofline": {
            "bound": "hbm",
            "achieved": r["hbm_gbs"],
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": r["hbm_frac"],
            "traffic": traffic,
            "kernel": r["kernel"],
            "kernel_avg_ms": r["kernel_avg_ms"],
            "frames_per_launch": r["frames_per_launch"],
            "launches": r["launches"],
            "kernel_ms_per_frame": r["kernel_ms_per_frame"],
            "frame_period_ms": r["frame_period_ms"],
            "kernel_avg_ms_launch_events": r["kernel_avg_ms_launch_events"],
            "kernel_avg_source": ("HIP events around the timed region on the launch stream / launches (one launch "
                                  "in flight, launches back to back: the launches alone on the GPU, as rocprofv3's "
                                  "kernel trace of the same command); kernel_avg_ms_launch_events = an untimed "
                                  "second pass of the same launches with an event pair around each")
            if isolated else "sampled HIP event pairs of overlapping launches (--inflight > 1)",
            "note": "algorithmic bytes = 4 B framebuffer store per pixel x frames per launch; traffic = PMC "
                    "FETCH_SIZE x 2 + WRITE_SIZE per launch (profiles/pmc_traffic.json); the path is "
                    "FP32-VALU-bound (roofline_valu)",
        },
        "roofline_valu": {
            "bound": "valu",
            # issued VALU lane-ops (PMC SQ_INSTS_VALU x 64) per frame over the kernel time per frame
            "achieved": valu_frame * 64 / kernel_frame_s / 1e12 if valu_frame else None,
            "peak": VALU_PEAK_TOPS,
            "unit": "TOP/s",
            "frac": valu_frame * 64 / kernel_frame_s / 1e12 / VALU_PEAK_TOPS if valu_frame else None,
            "brute_force_equiv": r["f_alg"] / steps / kernel_frame_s / 1e12,
            "note": "achieved = issued VALU lane-ops per frame (profiles/pmc_traffic.json SQ_INSTS_VALU x 64) / "
                    "kernel time per frame; brute_force_equiv = 24 ops per sphere test + 17 per plane test over "
                    "every primitive (SURVEY.md 8d) / kernel time -- above peak where culling skips tests",
        },
        "cpu_baseline": None,
        "host_ms_per_step": m["host_s"] * 1e3,
    }
    if not args.no_tick:
        # Work actually executed (diagnostic kernels, one frame, untimed) beside the nominal counts:
        # Mray/s counts SURVEY 8(d)'s visible-path rays, some of whose shadow tests are skipped
        w = ctx.count_work(W, H)
        nominal = w["primary_rays"] + w["reflect_rays"] + w["shadow_rays"]
        out["work_per_frame"] = dict(w, rays=nominal, rays_match_timed_run=nominal == r["rays_per_frame"],
                                     note="nominal counts (SURVEY.md 8d: every primitive of every visible-path ray) "
                                          "vs *_run = exact tests / shadow rays the kernel executed (skipped: shadow "
                                          "tests that cannot change the pixel, culled spheres)")
        out.update(tick_rates(ctx, W, H, torch))
        # the single-frame dispatch order the library measured and kept for this scene (rt_dispatch_order;
        # RT_DISPATCH_ORDER fixes it): single_launch_fps depends on it
        out["dispatch_order"] = ctx.dispatch_order()
        tick_cfgs = [c for c in (x.strip() for x in args.tick_configs.split(",")) if c]
        if tick_cfgs:
            out["tick_by_config"] = plugin_ticks(ctx, tick_cfgs, scenes)
            out["tick_by_config"]["note"] = ("plugin-path Tick() per config, one GPU: tick_fps = rt_render (synchronous, "
                                             "large frames traced in chunks, each chunk's PCIe copy by the copy engine "
                                             "on a second stream under the next chunk's trace), tick_async_fps = "
                                             "rt_render_async two frames deep; d2h_gbs = frame bytes x fps; median of 3 "
                                             "runs of 20 frames; work counters off (the display loop's setting)")
            ctx.set_scene(sc)
    also = [c for c in (x.strip() for x in args.also.split(",")) if c and c.upper() != sc.name.upper()]
    if also:
        out["also"] = {}
        for name in also:
            sc2 = scenes.config(name)
            ctx.set_scene(sc2)
            r2 = single_summary(sc2, measure_single(ctx, sc2, args, torch, abi, steps, args.warmup), steps)
            out["also"][sc2.name] = {k: r2[k] for k in ("value", "unit", "ms_per_step", "fps", "rays_per_frame",
                                                        "workload", "kernel", "kernel_avg_ms", "kernel_ms_per_frame",
                                                        "frames_per_launch", "launches", "hbm_frac")}
            if not args.no_tick:  # the same config one frame per launch (a display loop's shape, counters off)
                frames_lone = max(16, min(200, int(0.03 / max(r2["ms_per_step"] / 1e3, 1e-6))))
                out["also"][sc2.name]["lone_frame"] = lone_frame_rate(ctx, sc2.width, sc2.height, torch, frames_lone)
            # VALU issue (the binding resource) from the committed PMC summary of this config, as for the line
            pmc2 = load_pmc(args.pmc, sc2.name, 1)
            v2 = (pmc2.get("counters") or {}).get("SQ_INSTS_VALU") if pmc2 else None
            if v2:
                per_frame = v2 / (pmc2.get("frames_per_launch") or 1)
                out["also"][sc2.name]["valu_frac"] = (per_frame * 64 / (r2["kernel_ms_per_frame"] / 1e3) / 1e12
                                                      / VALU_PEAK_TOPS)
    if not args.no_cpu_baseline:
        # the bench config, then the other 1080p config (C2 beside C3: BASELINE.md's "C2/C3 at 1920x1080
        # beside the GPU"), C1 (BASELINE configs[0]) and the verbatim reference scene beside it
        other = "C2" if sc.name.upper() == "C3" else "C3"
        o_sc = scenes.config(other)
        o_rays = out.get("also", {}).get(other, {}).get("rays_per_frame")
        cpu_samples = [(sc, r["rays_per_frame"], 0.4)]
        if sc.name.upper() != other:
            cpu_samples.append((o_sc, o_rays, 0.25))
        cpu_samples += [(scenes.config("C1"), None, 0.15), (scenes.reference(512, 512), None, 0.2)]
        out["cpu_baseline"] = cpu_baseline(cpu_samples, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
