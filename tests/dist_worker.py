"""Worker for the multi-process (gloo, CPU) tests of raytracer_hip.dist.

Each rank traces only its own interleaved row bands -- with the CPU oracle standing in for
rt_render_bands, since there is no GPU here -- packs them into its slot, the slots are
gathered to rank 0 with torch.distributed (gloo), and rank 0 reassembles the frame with the
host mirror of rt_scatter_bands and compares it with the oracle's full frame.
"""
import os
import sys


def run(rank, world, port, cfg, width, height, band_rows, result_path):
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "uu-infogr-raytracer_amd"), os.path.join(root, "oracle"), here]
    import numpy as np
    import torch
    import torch.distributed as dist

    import pyoracle
    from raytracer_hip import scenes
    from raytracer_hip.dist import BandGather, RowBands, scatter_host

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = scenes.config(cfg).resized(width, height)
        rb = RowBands(width, height, band_rows, rank, world)
        g = BandGather(rb, "cpu")
        local = g.local.numpy().reshape(-1, width)
        for l0, y0, n in rb.row_spans():
            rows, _ = pyoracle.render(sc, pyoracle.MODE_NEAREST, 2, rows=(y0, y0 + n))
            local[l0:l0 + n] = rows
        parts = g.gather()
        ok = torch.tensor([1], dtype=torch.int32)
        if rank == 0:
            frame = scatter_host([p.numpy() for p in parts], width, height, band_rows)
            full, _ = pyoracle.render(sc, pyoracle.MODE_NEAREST, 2)
            same = bool(np.array_equal(frame, full))
            ok[0] = int(same)
            with open(result_path, "w") as f:
                f.write("ok" if same else f"mismatch {int((frame != full).sum())}")
        dist.broadcast(ok, 0)
        assert ok.item() == 1
    finally:
        dist.destroy_process_group()


def run_pipelined(rank, world, port, cfg, width, height, band_rows, frames, result_path):
    """Consecutive frames (a different camera yaw each) through PipelinedBandGather; rank 0
    checks every reassembled frame against the oracle's full frame for that camera."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "uu-infogr-raytracer_amd"), os.path.join(root, "oracle"), here]
    import numpy as np
    import torch
    import torch.distributed as dist

    import pyoracle
    from raytracer_hip import scenes
    from raytracer_hip.dist import PipelinedBandGather, RowBands, scatter_host

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        base = scenes.config(cfg).resized(width, height)

        def scene_for(k):
            sc = base.resized(width, height)
            sc.camera = ((0.0, 0.0, 0.0), 0.05 * k - 0.1, 0.02 * k)
            return sc

        rb = RowBands(width, height, band_rows, rank, world)
        pg = PipelinedBandGather(rb, "cpu")
        got = []
        for k in range(frames):
            local = pg.buffer().numpy().reshape(-1, width)
            local[:] = -3
            for l0, y0, n in rb.row_spans():
                rows, _ = pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2, rows=(y0, y0 + n))
                local[l0:l0 + n] = rows
            done = pg.submit()
            if done is not None and rank == 0:
                got.append(scatter_host([t.numpy() for t in done], width, height, band_rows))
        done = pg.drain()
        if rank == 0:
            got.append(scatter_host([t.numpy() for t in done], width, height, band_rows))
            bad = []
            for k, frame in enumerate(got):
                full, _ = pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2)
                if not np.array_equal(frame, full):
                    bad.append(k)
            with open(result_path, "w") as f:
                f.write("ok" if len(got) == frames and not bad else f"bad frames {bad} of {len(got)}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def run_batched(rank, world, port, cfg, width, height, band_rows, frames, per_batch, result_path):
    """bench.py's N>1 step: F frames per gather, RGB24 band sets, rank 0 reassembles every
    frame with the host mirror of rt_scatter_gathered and checks it against the oracle."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "uu-infogr-raytracer_amd"), os.path.join(root, "oracle"), here]
    import ctypes
    import numpy as np
    import torch.distributed as dist

    import pyoracle
    from raytracer_hip import scenes
    from raytracer_hip.dist import BatchedBandGather, RowBands, pack_rgb24, scatter_gathered_host

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        base = scenes.config(cfg).resized(width, height)

        def scene_for(k):
            sc = base.resized(width, height)
            sc.camera = ((0.0, 0.0, 0.0), 0.04 * k - 0.1, -0.02 * k)
            return sc

        rb = RowBands(width, height, band_rows, rank, world)
        g = BatchedBandGather(rb, "cpu", frames_per_batch=per_batch)
        got = []

        def consume(done):
            for buf, n in done:
                host = buf.numpy()
                for f in range(n):
                    got.append(scatter_gathered_host(host[f * g.slot_bytes:], g.rank_stride, width, height,
                                                     band_rows, world))

        for k in range(frames):
            ptr = g.frame_buffer()
            dst = (ctypes.c_uint8 * g.slot_bytes).from_address(ptr)
            slot = np.frombuffer(dst, dtype=np.uint8)
            slot[:] = 0xEE
            for l0, y0, n in rb.row_spans():
                rows, _ = pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2, rows=(y0, y0 + n))
                b = pack_rgb24(rows)
                slot[l0 * width * 3:l0 * width * 3 + b.size] = b
            done = g.commit()
            if done is not None and rank == 0:
                consume([done])
        rest = g.drain()
        if rank == 0:
            consume(rest)
            bad = [k for k, fr in enumerate(got)
                   if not np.array_equal(fr, pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2)[0])]
            with open(result_path, "w") as f:
                f.write("ok" if len(got) == frames and not bad else f"bad frames {bad} of {len(got)}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def run_tiles(rank, world, port, cfg, width, height, band_rows, frames, per_batch, result_path, rank0_codec=False,
              compositor=False, speculate=0, spec_after_drain=False, tail=0):
    """bench.py's default N>1 step: F frames per batch, tile-encoded band sets (host mirror of
    rt_encode_bands), size all_reduce + gather, rank 0 decodes every frame (host mirror of
    rt_decode_gathered) and checks it against the oracle."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "uu-infogr-raytracer_amd"), os.path.join(root, "oracle"), here]
    import numpy as np
    import torch
    import torch.distributed as dist

    import pyoracle
    from raytracer_hip import scenes, tilecodec
    from raytracer_hip.dist import RowBands, TileBandGather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        base = scenes.config(cfg).resized(width, height)

        def scene_for(k):
            sc = base.resized(width, height)
            sc.camera = ((0.0, 0.0, 0.0), 0.04 * k - 0.1, -0.02 * k)
            return sc

        # compositor: ranks 1..N-1 are band ranks 0..N-2 of a band world of N-1, rank 0 only decodes;
        # with `tail` rows, ranks 1..N-1 cover rows [0, H - tail) and rank 0 renders the last `tail` rows
        brank, bworld = (max(0, rank - 1), world - 1) if compositor else (rank, world)
        hb = height - tail  # the band geometry's rows
        rb = RowBands(width, hb, band_rows, brank, bworld)
        got = {}
        pending = {}  # batch -> (frame ring, frames) decoded, not yet read out of its ring

        def encode(raw, n, wire, size, _stream):
            b = tilecodec.encode(raw.numpy()[:n * rb.slot_elems], width, hb, band_rows, brank, bworld, n)
            wire.numpy()[:len(b)] = np.frombuffer(b, dtype=np.uint8)
            size[0] = len(b)

        def decode(recv, rank_stride, n, frames_, _stream, first_rank):
            # (a speculative batch that outgrew its gather is decoded twice: the later decode stands,
            # so a batch's frames are read out of the ring only before the ring is rendered again)
            host = recv.numpy()
            fr = frames_.numpy().reshape(-1, height, width)
            for r in range(first_rank, bworld):  # (rows [0, hb) of each frame)
                tilecodec.decode_into(fr[:n, :hb], host[r * rank_stride:(r + 1) * rank_stride], width, hb,
                                      band_rows, r, bworld)
            pending[g.decode_batch] = (fr, n)

        def read_out(upto):
            for b in sorted(x for x in pending if x <= upto):
                fr, n = pending.pop(b)
                for f in range(n):
                    got[b * g.F + f] = fr[f].copy()
                    fr[f] = -7  # the ring slot is reused: stale pixels must not pass

        g = TileBandGather(rb, "cpu", per_batch, lambda n: tilecodec.layout(width, hb, band_rows, bworld, n),
                           encode, decode, rank0_codec=rank0_codec, compositor=compositor, phys_rank=rank,
                           phys_world=world, tail_rows=tail)
        if rank == 0:
            for ring in g.frames:
                ring.fill_(-7)
        for k in range(frames):
            if k % g.F == 0:
                if speculate and k == 2 * g.F:  # the sizes of the first batches are known by now
                    if spec_after_drain:  # as bench.py: the warm-up drained, the pipeline is empty
                        g.drain()
                    g.set_capacity(speculate)
                g.begin_batch()
                read_out(k // g.F - 3)  # this batch renders into the ring of batch b-3
            if g.idle:  # the compositor rank renders nothing
                g.commit()
                continue
            dst = g.target().numpy()
            if g.direct and tail:  # rank 0 renders the frame's last `tail` rows into its frame
                dst = dst.reshape(height, width)
                rows, _ = pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2, rows=(hb, height))
                dst[hb:height] = rows
            elif g.direct:  # rank 0 renders its bands into their frame rows
                dst = dst.reshape(height, width)
                for l0, y0, n in rb.row_spans():
                    rows, _ = pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2, rows=(y0, y0 + n))
                    dst[y0:y0 + n] = rows
            else:
                dst[:] = 0x5A5A5A  # rows this rank does not own must not leak into the frame
                for l0, y0, n in rb.row_spans():
                    rows, _ = pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2, rows=(y0, y0 + n))
                    dst[l0 * width:(l0 + n) * width] = rows.reshape(-1)
            g.commit()
        g.drain()
        read_out(frames)
        if speculate and speculate < 1 and spec_after_drain:  # (only a batch that finds the pipeline
            assert g.redone > 0, "a margin below 1 must force a gather at the real size"  # empty guesses)
            # a redone batch was decoded twice and the second decode stands
            assert sum(1 for n in g.decodes_of.values() if n == 2) == g.redone, g.decodes_of
        assert not g.provisional, f"batches left provisional after drain: {g.provisional}"
        if rank == 0:
            bad = [k for k in range(frames)
                   if k not in got or not np.array_equal(got[k], pyoracle.render(scene_for(k), pyoracle.MODE_NEAREST, 2)[0])]
            with open(result_path, "w") as f:
                f.write("ok" if not bad else f"bad frames {bad} of {len(got)}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def run_timed_attempts(rank, world, port, result_path):
    """bench.timed_attempts at world `world` over gloo with a speculative gather forced too short
    (the all-reduced wire size exceeds the speculative size on every rank, as a margin below 1
    makes it): every rank repeats the region once, and the counters afterwards (rays, wire bytes,
    redone batches) are those of the reported, second attempt alone."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "uu-infogr-raytracer_amd"), here]
    import torch
    import torch.distributed as dist

    import bench
    from raytracer_hip import tilecodec
    from raytracer_hip.dist import RowBands, TileBandGather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W, H, br, steps = 64, 32, 8, 4
        rb = RowBands(W, H, br, rank, world)
        tg = TileBandGather(rb, "cpu", steps, lambda n: tilecodec.layout(W, H, br, world, n), None, None,
                            rank0_codec=True)
        tg.capacity_per_frame = 150.0  # speculative gather: 600 bytes for the 4-frame batch

        class Ctx:
            rays = 0

            def reset_stats(self):
                self.rays = 0

        ctx = Ctx()
        rays_per_attempt = 1000 * steps

        def region():
            ctx.rays += rays_per_attempt
            size = torch.tensor([500 + 400 * rank], dtype=torch.int64)  # this rank's wire
            dist.all_reduce(size, op=dist.ReduceOp.MAX)
            if tg.defer_checks:  # speculative: ships 600 bytes, the size is reduced and checked afterwards
                tg.size[0].fill_(500 + 400 * rank)  # this rank's wire; check_deferred reduces the maximum
                tg.provisional.add(tg.batch)
                tg.pending_checks.append((tg.batch, steps, 600, 0))
                tg.bytes_sent += 600
            else:  # exact size
                tg.bytes_sent += (int(size) + 7) // 8 * 8
            tg.batch += 1
            return 0.5, 0.1

        logs = []
        timing, repeats = bench.timed_attempts(ctx, tg, True, region, dist.barrier, logs.append)
        want_bytes = (500 + 400 * (world - 1) + 7) // 8 * 8
        good = (timing == (0.5, 0.1) and repeats == 1 and ctx.rays == rays_per_attempt
                and tg.bytes_sent == want_bytes and tg.redone == 0 and tg.deferred_failed == 1
                and tg.abandoned == {0} and not tg.provisional and not tg.defer_checks and len(logs) == 1)
        ok = torch.tensor([int(good)], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if rank == 0:
            with open(result_path, "w") as f:
                f.write("ok" if int(ok) else "mismatch")
        assert good, (timing, repeats, ctx.rays, tg.bytes_sent, tg.redone, tg.deferred_failed, tg.abandoned)
    finally:
        dist.destroy_process_group()


def run_library_collectives(rank, world, port, probe_fails, uid_fails, init_fails, result_path):
    """LibraryCollectives' construction protocol over gloo with a stand-in context: whichever rank
    cannot load RCCL (probe_fails) or make the id (uid_fails: rank 0), every rank reaches the same
    collectives and takes the same decision; rt_comm_init is entered by all ranks or by none."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "uu-infogr-raytracer_amd"), here]
    import torch
    import torch.distributed as dist

    from raytracer_hip.dist import CommUnavailable, LibraryCollectives

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        class Ctx:
            inits = []

            def comm_probe(self):
                return rank not in probe_fails

            def comm_unique_id(self):
                if uid_fails:
                    raise RuntimeError("ncclGetUniqueId failed")
                return bytes(range(128))

            def comm_init(self, w, r, uid):
                self.inits.append((w, r, uid))
                if r in init_fails:
                    raise RuntimeError("ncclCommInitRank failed")

        def agree_min(v):
            t = torch.tensor([v], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return int(t)

        ctx = Ctx()
        outcome = "built"
        try:
            LibraryCollectives(ctx, rank, world, lambda t: dist.broadcast(t, src=0), agree_min, device="cpu")
        except CommUnavailable:
            outcome = "unavailable"
        except RuntimeError:
            outcome = "init-failed"
        chosen = agree_min(1 if outcome == "built" else 0)  # bench.py's agreement afterwards
        expect = "unavailable" if (probe_fails or uid_fails) else ("init-failed" if rank in init_fails else "built")
        good = outcome == expect and chosen == (0 if (probe_fails or uid_fails or init_fails) else 1)
        good = good and (ctx.inits == [] if expect == "unavailable" else ctx.inits == [(world, rank, bytes(range(128)))])
        ok = torch.tensor([int(good)], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if rank == 0:
            with open(result_path, "w") as f:
                f.write("ok" if int(ok) else "mismatch")
    finally:
        dist.destroy_process_group()
