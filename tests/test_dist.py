"""Multi-rank data path (interleaved row bands + gather to rank 0 + reassembly) with
world_size 2 and 3 under torch.distributed gloo on CPU, plus the band-layout arithmetic."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from raytracer_hip.dist import RowBands, bands_of, scatter_host


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("H,band_rows,world", [(1080, 8, 2), (1080, 8, 8), (117, 5, 8), (7, 8, 4), (100, 1, 3),
                                               (4320, 8, 8)])
def test_band_layout_covers_every_row_once(H, band_rows, world):
    W = 3
    seen = np.zeros(H, dtype=int)
    for r in range(world):
        rb = RowBands(W, H, band_rows, r, world)
        assert rb.n_bands <= rb.max_bands and rb.max_bands - rb.n_bands <= 1
        for l0, y0, n in rb.row_spans():
            assert rb.global_row(l0) == y0
            seen[y0:y0 + n] += 1
    assert (seen == 1).all()
    assert sum(bands_of(H, band_rows, r, world) for r in range(world)) == -(-H // band_rows)


def test_scatter_host_roundtrip():
    W, H, br, world = 13, 29, 4, 3
    frame = np.arange(W * H, dtype=np.int32).reshape(H, W)
    parts = []
    for r in range(world):
        rb = RowBands(W, H, br, r, world)
        slot = np.full((rb.slot_elems // W, W), -5, dtype=np.int32)
        for l0, y0, n in rb.row_spans():
            slot[l0:l0 + n] = frame[y0:y0 + n]
        parts.append(slot.ravel())
    assert np.array_equal(scatter_host(parts, W, H, br), frame)


@pytest.mark.parametrize("world,cfg,w,h,band_rows", [(2, "C3", 64, 37, 8), (3, "REF", 48, 40, 5)])
def test_gloo_band_gather_reassembles_oracle_frame(tmp_path, world, cfg, w, h, band_rows):
    import dist_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    result = tmp_path / "result.txt"
    procs = [ctx.Process(target=dist_worker.run, args=(r, world, port, cfg, w, h, band_rows, str(result)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    assert result.read_text() == "ok"


@pytest.mark.parametrize("world,frames", [(2, 5), (3, 4)])
def test_gloo_pipelined_gather_keeps_frames_apart(tmp_path, world, frames):
    """Double-buffered gather (bench.py's N>1 step): every frame reassembles to its own oracle frame."""
    import dist_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    result = tmp_path / "result.txt"
    procs = [ctx.Process(target=dist_worker.run_pipelined,
                         args=(r, world, port, "C3", 48, 35, 4, frames, str(result))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    assert result.read_text() == "ok"


@pytest.mark.parametrize("world,frames,per_batch", [(2, 7, 3), (3, 5, 2), (2, 4, 4)])
def test_gloo_batched_rgb24_gather(tmp_path, world, frames, per_batch):
    """F frames per gather, RGB24 bands, one reassembly per frame (bench.py's N>1 step);
    the last batch may be partial."""
    import dist_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    result = tmp_path / "result.txt"
    procs = [ctx.Process(target=dist_worker.run_batched,
                         args=(r, world, port, "C3", 40, 29, 4, frames, per_batch, str(result))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    assert result.read_text() == "ok"


def test_scatter_gathered_host_matches_scatter_host():
    from raytracer_hip.dist import pack_rgb24, scatter_gathered_host
    W, H, br, world = 11, 23, 3, 4
    frame = (np.arange(W * H, dtype=np.int32) * 0x01F3A7) & 0xFFFFFF
    frame = frame.reshape(H, W)
    for bpp in (3, 4):
        stride = 1000
        buf = np.zeros(world * stride, dtype=np.uint8)
        for r in range(world):
            rb = RowBands(W, H, br, r, world)
            for l0, y0, n in rb.row_spans():
                rows = frame[y0:y0 + n]
                b = pack_rgb24(rows) if bpp == 3 else rows.astype(np.int32).view(np.uint8).reshape(-1)
                buf[r * stride + l0 * W * bpp:r * stride + l0 * W * bpp + b.size] = b
        assert np.array_equal(scatter_gathered_host(buf, stride, W, H, br, world, bpp), frame)


@pytest.mark.parametrize("world,frames,per_batch,rank0_codec,compositor,speculate,after_drain",
                         [(2, 7, 3, False, False, 0, False), (3, 5, 2, False, False, 0, False),
                          (2, 9, 2, False, False, 0, False), (3, 7, 3, True, False, 0, False),
                          (3, 7, 3, False, True, 0, False), (4, 5, 2, False, True, 0, False),
                          (2, 4, 4, False, True, 0, False), (2, 9, 2, False, False, 1.25, False),
                          (3, 9, 2, False, True, 0.5, False), (2, 8, 2, True, False, 0.25, False),
                          (2, 5, 2, False, False, 0.25, True), (3, 9, 2, False, True, 1.25, True),
                          (3, 9, 2, True, False, 0.5, True),
                          # the driver's N = 8 shape: compositor, a short run as one batch after the
                          # warm-up drained the pipeline (speculative gather-first path)
                          (8, 5, 5, False, True, 1.25, True)])
def test_gloo_tile_encoded_gather(tmp_path, world, frames, per_batch, rank0_codec, compositor, speculate,
                                  after_drain, tail=0):
    """bench.py's default N>1 step: tile-encoded band sets, size all_reduce + gather, three-stage
    pipeline; every frame decodes to its own oracle frame, the last batch may be partial.  With
    `compositor` (bench.py at N >= 8) rank 0 traces nothing and decodes every band set.  With
    `speculate`, set_capacity(margin) is called after the first two batches: batches inside the
    pipeline keep their exact sizes.  With `after_drain` the pipeline is drained before the switch
    (as bench.py's warm-up): the next batch finds it empty and takes the speculative gather-first
    path (decode before the size check; margins below 1 force a second gather and decode at the
    reduced size); with 5 frames in batches of 2 that batch is the last, partial one, as in a
    short run."""
    import dist_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    result = tmp_path / "result.txt"
    procs = [ctx.Process(target=dist_worker.run_tiles,
                         args=(r, world, port, "C3", 43, 29, 4, frames, per_batch, str(result), rank0_codec,
                               compositor, speculate, after_drain, tail))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    assert result.read_text() == "ok"


@pytest.mark.parametrize("world,frames,per_batch,tail,speculate,after_drain",
                         [(2, 5, 2, 8, 0, False), (3, 7, 3, 4, 0, False), (4, 5, 2, 12, 0, False),
                          (8, 5, 5, 4, 1.25, True), (3, 9, 2, 8, 0.5, True), (4, 7, 7, 24, 1.25, True)])
def test_gloo_tile_gather_rank0_tail(tmp_path, world, frames, per_batch, tail, speculate, after_drain):
    """Rank 0's measured share (bench.py rank0_tail_rows): ranks 1..N-1 trace rows [0, H - tail) as a band
    world of N-1 and tile-encode them; rank 0 renders the last `tail` rows straight into its frames and
    decodes the others' -- every frame (29 rows: the band geometry's rows are cut at 29 - tail, not a
    multiple of the 8-row tile) equals the oracle's, including the driver's N = 8 one-batch speculative
    shape and a forced second gather (margin 0.5)."""
    test_gloo_tile_encoded_gather(tmp_path, world, frames, per_batch, False, True, speculate, after_drain, tail)


def test_deferred_size_check_decision():
    """TileBandGather.check_deferred (the one-batch bench run's size check after its closing sync):
    a speculative gather that sufficed makes its batch final; one that a wire outgrew keeps the batch
    provisional (ring_of refuses it) and asks the caller to repeat the run."""
    from raytracer_hip import tilecodec
    from raytracer_hip.dist import TileBandGather
    W, H, br = 64, 32, 8
    rb = RowBands(W, H, br, 0, 1)
    from raytracer_hip.dist import _Done
    g = TileBandGather(rb, "cpu", 4, lambda n: tilecodec.layout(W, H, br, 1, n), None, None, rank0_codec=True)
    g._size_reduce = lambda i: _Done()  # (world of one: the maximum over ranks is the rank's own size)
    g.provisional.update({0, 1})
    g.pending_checks = [(0, 4, 800, 0)]
    g.size[0].fill_(790)  # rounded up to 792 <= 800: the gather sufficed
    assert g.check_deferred() is True and 0 not in g.provisional and g.redone == 0
    g.pending_checks = [(1, 4, 800, 1)]
    g.size[1].fill_(801)
    assert g.check_deferred() is False and 1 not in g.provisional and 1 in g.abandoned
    assert g.redone == 0 and g.deferred_failed == 1
    assert g.pending_checks == [] and g.max_per_frame == 808 / 4
    with pytest.raises(RuntimeError):
        g.ring_of(1)
    # a deferred run longer than three batches: batch 3's encode would overwrite batch 0's size slot
    g.pending_checks = [(0, 4, 800, 0)]
    g.batch = 3
    with pytest.raises(RuntimeError, match="deferred size check"):
        g._stage_a(None, 4)
    assert g.batch == 3


def test_world_of_one_direct_rank_exchanges_nothing(monkeypatch):
    """A world of one rank that renders its bands straight into its frames (the one-GPU rehearsal of
    the default N > 1 path) has nothing to ship: its batches issue no size reduce, gather or decode,
    and every batch is final as traced.  With rank 0 through the codec (--rank0-codec) the exchange
    is still issued."""
    from raytracer_hip import tilecodec
    from raytracer_hip.dist import TileBandGather
    W, H, br, F = 64, 32, 8, 4
    rb = RowBands(W, H, br, 0, 1)
    g = TileBandGather(rb, "cpu", F, lambda n: tilecodec.layout(W, H, br, 1, n), None, None)
    assert g.solo and g.direct

    def no_exchange(*a, **k):
        raise AssertionError("a world of one direct rank issued an exchange")
    monkeypatch.setattr(g, "_size_reduce", no_exchange)
    monkeypatch.setattr(g, "_gather", no_exchange)
    monkeypatch.setattr(g, "_decode", no_exchange)
    for _ in range(3 * F):
        g.commit(None)
    g.drain(None)
    assert g.batch == 3 and g.decoded == 3 and g.bytes_sent == 0 and not g.provisional
    assert g.ring_of(2) is g.frames[2]
    codec = TileBandGather(rb, "cpu", F, lambda n: tilecodec.layout(W, H, br, 1, n), None, None, rank0_codec=True)
    assert not codec.solo


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_timed_region_repeat_counts_one_attempt(tmp_path, world):
    """bench.py's N>1 timed region with a speculative gather forced too short (every rank repeats the
    region, as `--spec-margin` < 1 makes it on GPUs): rays, wire bytes and redone batches reported
    afterwards are those of the repeated attempt alone, not the sum of both."""
    import dist_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    result = tmp_path / "result.txt"
    procs = [ctx.Process(target=dist_worker.run_timed_attempts, args=(r, world, port, str(result)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    assert result.read_text() == "ok"


@pytest.mark.parametrize("world,probe_fails,uid_fails,init_fails",
                         [(2, (), False, ()), (2, (1,), False, ()), (3, (0,), False, ()), (2, (), True, ()),
                          (3, (), False, (2,))])
def test_gloo_library_collectives_agree(tmp_path, world, probe_fails, uid_fails, init_fails):
    """bench.py's choice between the library's RCCL communicator and torch.distributed: a rank that
    cannot load RCCL, or a rank 0 that cannot make the unique id, makes every rank fall back without
    entering rt_comm_init (no rank left blocked in a collective the others skipped); an init failure
    on one rank makes every rank fall back through the agreement afterwards."""
    import dist_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    result = tmp_path / "result.txt"
    procs = [ctx.Process(target=dist_worker.run_library_collectives,
                         args=(r, world, port, probe_fails, uid_fails, init_fails, str(result)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    assert result.read_text() == "ok"
