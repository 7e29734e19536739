"""Isolated timings of the tile codec kernels on a traced frame (GPU box).

For world N (simulated in one process): each rank's band set of the frame is traced, then
encode (per rank, F frames per launch) and decode (all ranks, F frames) are timed alone with
HIP events, and the round trip is checked bit for bit.

    python tools/codec_bench.py --config C2 --worlds 1 2 8 --frames 8
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "uu-infogr-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 8])
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch

    from raytracer_hip import Context, abi, scenes, wire_layout
    from raytracer_hip.dist import RowBands
    sc = scenes.config(a.config)
    W, H, F, br = sc.width, sc.height, a.frames, 8
    ctx = Context(1)
    ctx.set_scene(sc)
    full = ctx.render(W, H).copy()
    s = torch.cuda.current_stream()
    for world in a.worlds:
        lay = wire_layout(W, H, br, world, F)
        stride = (lay.max_bytes + 255) // 256 * 256
        gathered = torch.zeros(world * stride, dtype=torch.uint8, device="cuda")
        sizes = torch.zeros(world, dtype=torch.int64, device="cuda")
        raws = []
        for r in range(world):
            rb = RowBands(W, H, br, r, world)
            raw = torch.zeros(F * rb.slot_elems, dtype=torch.int32, device="cuda")
            for f in range(F):
                ctx.render_bands_ex(W, H, br, r, world, raw[f * rb.slot_elems:].data_ptr(), abi.RT_BANDS_INT32,
                                    s.cuda_stream)
            raws.append((rb, raw))
        frames = torch.zeros(F * W * H, dtype=torch.int32, device="cuda")

        def enc(r):
            rb, raw = raws[r]
            ctx.encode_bands(W, H, br, r, world, raw.data_ptr(), rb.slot_elems, F, gathered[r * stride:].data_ptr(),
                             sizes[r:].data_ptr(), s.cuda_stream)

        def dec():
            ctx.decode_gathered(W, H, br, world, gathered.data_ptr(), stride, F, frames.data_ptr(), W * H,
                                s.cuda_stream)

        for _ in range(3):
            enc(0)
            dec()
        for r in range(world):
            enc(r)
        dec()
        torch.cuda.synchronize()
        ok = all(np.array_equal(frames[f * W * H:(f + 1) * W * H].cpu().numpy().reshape(H, W), full) for f in range(F))
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(s)
        for _ in range(a.reps):
            enc(0)
        e1.record(s)
        for _ in range(a.reps):
            dec()
        e2.record(s)
        torch.cuda.synchronize()
        enc_us = e0.elapsed_time(e1) * 1e3 / a.reps / F
        dec_us = e1.elapsed_time(e2) * 1e3 / a.reps / F
        wire = sizes.cpu().numpy()
        print(f"{a.config} world {world}: encode (rank 0's band set) {enc_us:.2f} us/frame, decode (all ranks) "
              f"{dec_us:.2f} us/frame; wire bytes/frame/rank {wire.max() / F:.0f} (rgb24 {3 * raws[0][0].slot_elems}); "
              f"roundtrip {'bit-exact' if ok else 'MISMATCH'}", flush=True)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
