"""Row-band sharding of a frame across ranks (one process per GPU), SURVEY.md 8(e).

Pixels are independent, so a frame is split into interleaved bands of `band_rows` rows:
band b goes to rank b % world (sky rows are nearly free, contiguous tiles would be badly
imbalanced).  Each rank traces its bands packed one after the other into a slot of
`max_bands * band_rows * W` int32 (ranks with one band fewer leave the tail of the slot
unused), the slots are gathered to rank 0 -- torch.distributed backend "nccl" is RCCL on
ROCm, point-to-point over xGMI -- and rank 0 scatters each slot back into the row-major
frame (rt_scatter_bands on the GPU; `scatter_host` below is its host mirror).

The same code runs under backend "gloo" on CPU tensors for the multi-process tests.
"""
from __future__ import annotations

import numpy as np


def bands_of(height: int, band_rows: int, first: int, step: int) -> int:
    """Number of bands b = first, first+step, ... with b*band_rows < height."""
    total = (height + band_rows - 1) // band_rows
    return (total - 1 - first) // step + 1 if first < total else 0


class RowBands:
    """This rank's share of a W x H frame."""

    def __init__(self, width: int, height: int, band_rows: int, rank: int, world: int):
        if band_rows <= 0 or world <= 0 or not 0 <= rank < world:
            raise ValueError("bad band layout")
        self.width, self.height, self.band_rows = width, height, band_rows
        self.rank, self.world = rank, world
        self.n_bands = bands_of(height, band_rows, rank, world)
        self.max_bands = bands_of(height, band_rows, 0, world)
        self.slot_elems = max(1, self.max_bands) * band_rows * width
        self.pixels = self.n_bands * band_rows * width  # traced by this rank (incl. rows past H)

    def global_row(self, local_row: int) -> int:
        """Frame row of packed local row `local_row` (may be >= height in the last band)."""
        band = self.rank + (local_row // self.band_rows) * self.world
        return band * self.band_rows + local_row % self.band_rows

    def row_spans(self):
        """[(local_row0, frame_row0, n_rows)] of every band of this rank, clipped to the frame."""
        out = []
        for k in range(self.n_bands):
            y0 = (self.rank + k * self.world) * self.band_rows
            n = min(self.band_rows, self.height - y0)
            out.append((k * self.band_rows, y0, n))
        return out


def pack_rgb24(pixels) -> np.ndarray:
    """Host mirror of RT_BANDS_RGB24: int32 0x00RRGGBB -> bytes B, G, R per pixel."""
    v = np.ascontiguousarray(pixels, dtype=np.int32).reshape(-1).view(np.uint8).reshape(-1, 4)
    return np.ascontiguousarray(v[:, :3]).reshape(-1)


def scatter_gathered_host(buf, rank_stride: int, width: int, height: int, band_rows: int, world: int,
                          bpp: int = 3) -> np.ndarray:
    """Host mirror of rt_scatter_gathered: rank r's band set at byte r * rank_stride of buf."""
    buf = np.asarray(buf, dtype=np.uint8).reshape(-1)
    frame = np.full((height, width), -1, dtype=np.int32)
    for y in range(height):
        b = y // band_rows
        r, k = b % world, b // world
        o = r * rank_stride + ((k * band_rows + y % band_rows) * width) * bpp
        row = buf[o:o + width * bpp].reshape(width, bpp)
        if bpp == 4:
            frame[y] = row.view(np.int32).reshape(-1)
        else:
            frame[y] = row[:, 0].astype(np.int32) | (row[:, 1].astype(np.int32) << 8) | (row[:, 2].astype(np.int32) << 16)
    return frame


def scatter_host(parts, width: int, height: int, band_rows: int) -> np.ndarray:
    """Host mirror of rt_scatter_bands for every rank's gathered slot (rank order)."""
    world = len(parts)
    frame = np.full((height, width), -1, dtype=np.int32)
    for rank, part in enumerate(parts):
        rb = RowBands(width, height, band_rows, rank, world)
        img = np.asarray(part).reshape(-1, width)
        for l0, y0, n in rb.row_spans():
            frame[y0:y0 + n] = img[l0:l0 + n]
    return frame


class BandGather:
    """Gather of every rank's band slot to rank 0 (torch.distributed, RCCL on ROCm GPUs)."""

    def __init__(self, rb: RowBands, device, dtype=None):
        import torch
        self.rb = rb
        dtype = dtype or torch.int32
        self.local = torch.zeros(rb.slot_elems, dtype=dtype, device=device)
        self.parts = [torch.empty_like(self.local) for _ in range(rb.world)] if rb.rank == 0 else None

    def gather(self):
        import torch.distributed as dist
        dist.gather(self.local, self.parts, dst=0)
        return self.parts


class PipelinedBandGather:
    """Double-buffered gather: frame k's gather overlaps frame k+1's trace.

    Per frame:  buf = pg.buffer()  -> trace this rank's bands into `buf`
                done = pg.submit() -> starts the gather of `buf` (async), then waits for
                                      the previous frame's gather and returns its slots
                                      (rank 0; None elsewhere / on the first frame)
    and finally `pg.drain()` returns the last frame's slots.

    Ordering on GPUs (ProcessGroupNCCL): the collective waits for the current stream's work
    enqueued before it (the trace of its buffer); `wait()` makes the current stream wait for
    the collective.  The wait for gather k is issued after trace k+1 was enqueued (overlap)
    and before trace k+2 reuses gather k's buffer, and rank 0 consumes gather k's slots
    after that wait; gather k+2 into the same slots is ordered after that consumption.
    """

    def __init__(self, rb: RowBands, device, depth: int = 2):
        import torch
        self.rb = rb
        self.depth = depth
        self.local = [torch.zeros(rb.slot_elems, dtype=torch.int32, device=device) for _ in range(depth)]
        self.parts = [[torch.empty_like(self.local[0]) for _ in range(rb.world)] if rb.rank == 0 else None
                      for _ in range(depth)]
        self.frame = 0
        self.pending = None  # (work, slot index)

    def buffer(self):
        return self.local[self.frame % self.depth]

    def submit(self):
        import torch.distributed as dist
        i = self.frame % self.depth
        work = dist.gather(self.local[i], self.parts[i], dst=0, async_op=True)
        done = None
        if self.pending is not None:
            pw, pi = self.pending
            pw.wait()
            done = self.parts[pi]
        self.pending = (work, i)
        self.frame += 1
        return done

    def drain(self):
        if self.pending is None:
            return None
        pw, pi = self.pending
        pw.wait()
        self.pending = None
        return self.parts[pi]


class BatchedBandGather:
    """F frames per RCCL gather, double-buffered (bench.py's N > 1 step).

    Each rank renders frame k's bands (RT_BANDS_RGB24 by default: 3 bytes per pixel) into
    slot k % F of the current batch buffer; after F frames one gather moves the whole batch to
    rank 0 -- one collective's latency per F frames -- while the next batch is traced.  On
    rank 0 the gathered buffer holds rank r's batch at r * rank_stride (rank_stride =
    F * slot_bytes), so frame f of the batch is reassembled by ONE rt_scatter_gathered
    launch from offset f * slot_bytes with rank stride rank_stride.

        buf = g.frame_buffer()   -> device pointer for this rank's frame k
        done = g.commit()        -> after frame k; (gathered tensor, n_frames) of the batch
                                    completed earlier (rank 0) or None
        done = g.drain()         -> at the end: submits a partial batch, returns what is left
    Ordering on GPUs (ProcessGroupNCCL): a gather waits for the current stream's earlier
    work (the traces of its batch); waiting on it makes the current stream wait for the
    collective, which is issued after the next batch's traces were enqueued and before the
    buffer is reused (depth 2).
    """

    def __init__(self, rb: RowBands, device, frames_per_batch: int = 4, bpp: int = 3, depth: int = 2):
        import torch
        self.rb, self.F, self.bpp, self.depth = rb, max(1, frames_per_batch), bpp, depth
        raw = max(1, rb.max_bands) * rb.band_rows * rb.width * bpp
        self.slot_bytes = (raw + 255) // 256 * 256
        self.rank_stride = self.F * self.slot_bytes
        self.local = [torch.zeros(self.rank_stride, dtype=torch.uint8, device=device) for _ in range(depth)]
        self.gathered = ([torch.empty(rb.world * self.rank_stride, dtype=torch.uint8, device=device)
                          for _ in range(depth)] if rb.rank == 0 else [None] * depth)
        self.k = 0          # frames rendered
        self.batch = 0      # batches submitted
        self.pending = None  # (work, buffer index, n_frames)

    def frame_buffer(self) -> int:
        b = self.local[self.batch % self.depth]
        return b.data_ptr() + (self.k % self.F) * self.slot_bytes

    def _submit(self, n_frames: int):
        import torch.distributed as dist
        i = self.batch % self.depth
        n = n_frames * self.slot_bytes
        # every rank gathers the same n bytes (the same frame count); rank 0's list points
        # into its contiguous buffer at rank_stride intervals
        send = self.local[i][:n]
        glist = ([self.gathered[i][r * self.rank_stride:r * self.rank_stride + n] for r in range(self.rb.world)]
                 if self.rb.rank == 0 else None)
        work = dist.gather(send, glist, dst=0, async_op=True)
        done = None
        if self.pending is not None:
            pw, pi, pn = self.pending
            pw.wait()
            done = (self.gathered[pi], pn)
        self.pending = (work, i, n_frames)
        self.batch += 1
        return done

    def commit(self):
        self.k += 1
        if self.k % self.F == 0:
            return self._submit(self.F)
        return None

    def drain(self):
        out = []
        if self.k % self.F:
            d = self._submit(self.k % self.F)
            if d is not None:
                out.append(d)
            self.k += self.F - self.k % self.F  # next frame starts a fresh batch
        if self.pending is not None:
            pw, pi, pn = self.pending
            pw.wait()
            out.append((self.gathered[pi], pn))
            self.pending = None
        return out


class TileBandGather:
    """Tile-encoded band sets, F frames per batch, three-stage pipeline (bench.py's N > 1 step).

    Rendered frames are mostly flat, so shipping them to rank 0 raw (3-4 bytes per pixel)
    spends xGMI bandwidth on redundancy; each rank r > 0 tile-encodes its batch
    (rt_encode_bands, format in raytracer_hip/tilecodec.py) and rank 0 decodes the other ranks'
    wires straight into its frames (rt_decode_gathered, first_rank 1).  Rank 0 renders its own
    bands directly into the frames (RT_BANDS_FRAME): they never travel, so it neither encodes
    nor decodes them (`rank0_codec=True` routes them through the codec anyway -- the
    one-process rehearsal uses that to exercise it).  A wire's size varies with the image, and
    a gather moves the same count from every rank, so each batch costs two collectives:

        A  encode batch b into wire b % 3; all_reduce(MAX) of the wire sizes   (async)
        B  batch b-1: wait for its all_reduce, read the max size on the host, gather that
           many bytes of every rank's wire into rank 0's receive buffer (b-1) % 2  (async)
        C  batch b-2 (rank 0): wait for its gather, decode the wires into frame ring (b-2) % 3

    run at every batch boundary, so the host waits only for a size that was reduced one batch
    earlier while the GPU traces the current batch.  On GPUs the waits for collectives are put
    on two side streams (`comm`, `dec`), never on the trace streams; events order buffer reuse
    (wire b % 3 is re-encoded only after gather b completed, receive buffer b % 2 is
    overwritten only after decode b, rank 0 renders batch b into frame ring b % 3 only after
    decode b-3 filled it -- `begin_batch`).  With gloo on CPU tensors (tests) the same
    sequence runs synchronously.

    Speculative mode (`set_capacity`, bench.py after its warm-up) for a batch that finds the
    pipeline empty (a run's first batch -- all of a short run): its gather size is a guess (1.25 x
    the largest wire per frame so far), issued in stage A right behind the encode, the size reduce
    after it, and stage C decodes before it reads the reduced size -- neither the reduce nor the
    host's read-back sits between encode and decode.  A batch whose largest wire outgrew the
    guess is gathered again in full and decoded again (every rank sees the same reduced size, so
    all of them take part).  Batches inside a pipeline keep the exact size of stage B.

        g.begin_batch(streams)      -> before frame k when k % F == 0 (rank 0: ring reuse)
        dst = g.target(k)           -> rank 0 direct: int32 view of frame k's ring slot (render
                                       its bands there, RT_BANDS_FRAME); else this rank's raw
                                       band set of frame k (RT_BANDS_INT32)
        g.commit(main_stream)       -> after frame k was traced (stages at batch ends)
        g.drain()                   -> submit a partial last batch and finish every stage
    `encode(raw_batch, n_frames, wire, size_tensor, stream)` and
    `decode(gathered, rank_stride, n_frames, frames, stream, first_rank)` do the codec work (the
    HIP library on GPUs, the host mirror in tests).  Rank 0's decoded frames of batch b are in
    `frames[b % 3]` (F frames, row-major) once stage C of b has run (`ring_of`).

    Compositor mode (`compositor=True`; bench.py at N >= 8): rank 0 traces nothing and only
    assembles -- it decodes every band set of each frame, which ranks 1..N-1 trace as a band
    world of N-1 (`rb` is then the band geometry: band rank = rank - 1, band world = N - 1;
    `phys_rank`/`phys_world` are the process group's).  At N = 8 rank 0's own 1/8 share of a
    1080p frame (≈3 µs) plus the decode of the other 7/8 (≈2 µs) made it the slowest rank;
    without the trace the slowest rank traces and encodes 1/7.  Rank 0 still
    takes part in both collectives (size 0; its own gather slot is receive slot N-1, scratch).

    Rank 0's measured share (`tail_rows` > 0, with the compositor geometry): ranks 1..N-1 trace rows
    [0, H') of the frame (H' = H - tail_rows; `rb` is the band geometry of that H'-row frame, traced
    with the full frame's view: rt_set_view_height) and rank 0 renders the frame's last tail_rows rows
    itself, straight into its frames (whole bands: tail_rows a multiple of band_rows), beside decoding
    the others' -- a share sized so that its trace plus the decode take as long as the others' trace
    (bench.py rank0_tail_rows; tail_rows 0 is the compositor).  `frame_h` = H.
    """

    def __init__(self, rb: RowBands, device, frames_per_batch, layout_fn, encode, decode, rank0_codec=False,
                 compositor=False, phys_rank=None, phys_world=None, fused=False, coll=None, main_stream=None,
                 tail_rows=0):
        import torch
        self.rb, self.F, self.device = rb, max(1, frames_per_batch), torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.layout_fn, self.encode, self.decode = layout_fn, encode, decode
        self.compositor = bool(compositor)
        self.prank = rb.rank if phys_rank is None else int(phys_rank)
        self.pworld = rb.world if phys_world is None else int(phys_world)
        if self.compositor and (self.pworld != rb.world + 1 or (self.prank > 0 and rb.rank != self.prank - 1)):
            raise ValueError("compositor mode: the band world is N-1 and band rank = rank-1")
        if not self.compositor and (self.pworld != rb.world or self.prank != rb.rank):
            raise ValueError("band geometry and process group differ outside compositor mode")
        self.tail = int(tail_rows)
        if self.tail and (not self.compositor or rank0_codec or self.tail % rb.band_rows):
            raise ValueError("rank 0's tail rows: compositor geometry, whole bands, rank 0 outside the codec")
        self.root = self.prank == 0
        self.first_rank = 0 if (rank0_codec or self.compositor) else 1
        # rank 0 renders into its frames: its interleaved bands, or its tail rows
        self.direct = self.root and ((not rank0_codec and not self.compositor) or self.tail > 0)
        self.idle = self.root and self.compositor and not self.tail  # rank 0 only assembles
        # a world of one rank that renders straight into its frames has nothing to exchange: no size
        # reduce, gather or decode is issued (the one-GPU rehearsal of the default path then measures
        # the trace and the pipeline's bookkeeping alone)
        self.solo = self.direct and self.pworld == 1
        # fused: this rank traces its bands straight into the wire of the batch (rt_render_bands_tiles;
        # `wire_target`), and stage A's encode(None, ...) only finishes that wire (rt_finish_wire)
        self.fused = bool(fused) and not (self.direct or self.idle)
        self.slot_elems = rb.slot_elems
        lay = layout_fn(self.F)
        self.rank_stride = (int(lay.max_bytes) + 255) // 256 * 256
        self.raw = ([torch.zeros(self.F * self.slot_elems, dtype=torch.int32, device=self.device) for _ in range(2)]
                    if not (self.direct or self.idle or self.fused) else None)
        self.wire = [torch.zeros(self.rank_stride, dtype=torch.uint8, device=self.device) for _ in range(3)]
        self.size = [torch.zeros(1, dtype=torch.int64, device=self.device) for _ in range(3)]
        self.size_host = torch.zeros(3, dtype=torch.int64, pin_memory=self.cuda)
        # physical rank r's receive slot: r (compositor: its band rank r-1; rank 0's own: slot N-1)
        self.recv = ([torch.zeros(self.pworld * self.rank_stride, dtype=torch.uint8, device=self.device)
                      for _ in range(2)] if self.root else [None, None])
        self.frame_h = rb.height + self.tail  # (the frame's rows: the band geometry's and rank 0's tail)
        self.frame_elems = rb.width * self.frame_h
        self.frames = ([torch.zeros(self.F * self.frame_elems, dtype=torch.int32, device=self.device)
                        for _ in range(3)] if self.root else None)
        # coll (GPUs): the library's collectives (LibraryCollectives) issued on `main_stream`, the
        # stream that encodes and now also gathers and decodes -- no hops into and out of the
        # framework's collective stream; else torch.distributed, waited on two side streams
        self.coll = coll if self.cuda else None
        if self.cuda:
            if self.coll is not None:
                self.comm = self.dec = main_stream if main_stream is not None else torch.cuda.current_stream(self.device)
            else:
                self.comm, self.dec = torch.cuda.Stream(self.device), torch.cuda.Stream(self.device)
            self.enc_events = [torch.cuda.Event() for _ in range(4)]
        self.k = 0             # frames rendered
        self.batch = 0         # batches encoded
        self.stage_b = []      # [(batch, n_frames, all_reduce work)]
        self.stage_c = []      # [(batch, n_frames, gather work)]
        self.encoded_ev = {}   # batch -> event after its encode on the main stream (wire ready)
        self.gathered_ev = {}  # batch -> event after its gather (wire reusable)
        self.decoded_ev = {}   # batch -> event after its decode (receive buffer / frame ring reusable)
        self.decoded = 0       # batches decoded (rank 0)
        self.bytes_sent = 0    # wire bytes gathered per rank (sum over batches)
        self.max_per_frame = 0.0  # largest reduced wire size / frames of a batch seen so far
        self.capacity_per_frame = None  # speculative gather size (set_capacity); None = wait for the size
        self.redone = 0        # batches whose wire outgrew the speculative size (gathered again)
        self.decode_batch = -1  # the batch of the decode being issued
        # Speculative batches are decoded before their reduced size is known: until _stage_c has checked
        # it, the batch's ring and decoded_ev[b] are provisional (a wire cut short decoded stale payload
        # bytes).  Invariant: once _stage_c(b) returns, decoded_ev[b] is the event of the decode that
        # stands (a redo's second decode replaces the first one's event, which only the redo gather --
        # reader=b, the receive buffer's last reader -- waits on); ring_of refuses provisional batches.
        self.provisional = set()
        self.decodes_of = {}    # batch -> decodes issued (2 for a redone speculative batch)
        # defer_checks (GPUs; a run of at most three batches): a speculative batch's reduced size is read
        # back asynchronously instead of behind a host wait in the middle of the run, and the caller
        # checks it after its own synchronisation (check_deferred); a batch that outgrew its gather
        # then stays provisional and the caller repeats the run without speculation
        self.defer_checks = False
        self.pending_checks = []  # [(batch, n_frames, speculative bytes, size slot)]
        self.deferred_failed = 0  # deferred checks that failed (each made the caller repeat its run)
        self.abandoned = set()    # batches of a failed deferred check (ring_of refuses them)

    def set_capacity(self, margin=1.25):
        """From now on gather each batch with a speculative size -- `margin` x the largest wire per
        frame seen so far (every rank holds the same all-reduced sizes, so they agree without
        communicating) -- issued right behind the encode, before the size reduce.  The reduced size
        is checked after the batch's decode was issued: a batch whose largest wire exceeded the
        speculative size is gathered again at its real size and decoded again (every rank takes
        the same decision from the same reduced value)."""
        if self.max_per_frame > 0:
            while self.stage_b:  # batches whose size reduce is out: gathered at their real size first
                self._stage_b()
            self.capacity_per_frame = self.max_per_frame * margin

    def _read_size(self, i, work):
        import torch
        if self.cuda:
            with torch.cuda.stream(self.comm):
                work.wait()
                self.size_host[i:i + 1].copy_(self.size[i], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.comm)
            ev.synchronize()
        else:
            work.wait()
            self.size_host[i] = self.size[i][0]
        return (int(self.size_host[i]) + 7) // 8 * 8

    def _gather(self, b, i, n, reader=None):
        """Gather n bytes of every rank's wire i into receive buffer b % 2, after batch b's encode
        and after the decode of batch `reader` (default b-2, the buffer's previous batch) has read
        that buffer."""
        import torch
        import torch.distributed as dist
        j = b % 2
        reader = b - 2 if reader is None else reader
        glist = None
        if self.root:
            slot = [(r - 1) % self.pworld if self.compositor else r for r in range(self.pworld)]
            glist = [self.recv[j][q * self.rank_stride:q * self.rank_stride + n] for q in slot]
        if self.cuda:
            with torch.cuda.stream(self.comm):
                # The gather is issued on `comm`, which ProcessGroupNCCL orders it after: wire i
                # must be encoded (a speculative gather is issued without waiting for the size
                # reduce, so nothing else orders it after the encode)
                self.comm.wait_event(self.encoded_ev[b])
                if reader in self.decoded_ev:  # receive buffer j was last read by that decode
                    self.comm.wait_event(self.decoded_ev[reader])
                for old in [x for x in self.decoded_ev if x < b - 4]:
                    del self.decoded_ev[old]
                if self.coll is not None:
                    return self.coll.gather(self.wire[i], n, self.recv[j] if self.root else None, self.rank_stride,
                                            1 if self.compositor else 0, self.comm)
                return dist.gather(self.wire[i][:n], glist, dst=0, async_op=True)
        return dist.gather(self.wire[i][:n], glist, dst=0, async_op=True)

    def ring_of(self, batch):
        if batch in self.provisional:
            raise RuntimeError(f"batch {batch}: decoded speculatively, its size not yet checked")
        if batch in self.abandoned:
            raise RuntimeError(f"batch {batch}: its speculative gather was too short (run repeated)")
        return self.frames[batch % 3]

    def wire_target(self, k=None):
        """Fused mode: the wire that frame k's batch is traced into."""
        k = self.k if k is None else k
        if not self.fused:
            raise RuntimeError("wire_target needs fused mode")
        return self.wire[(k // self.F) % 3]

    def target(self, k=None):
        k = self.k if k is None else k
        if self.idle:
            raise RuntimeError("the compositor rank traces nothing")
        if self.fused:
            raise RuntimeError("fused mode: trace into wire_target()")
        if self.direct:
            o = (k % self.F) * self.frame_elems
            return self.frames[(k // self.F) % 3][o:o + self.frame_elems]
        o = (k % self.F) * self.slot_elems
        return self.raw[(k // self.F) % 2][o:o + self.slot_elems]

    def raw_frame(self, k=None):  # (the band set of a rank that encodes)
        return self.target(k)

    def begin_batch(self, streams=()):
        """Before the first frame of a batch: rank 0's frame ring of this batch was last filled
        by the decode of batch b-3, which must finish before the ring is rendered into again."""
        b = self.k // self.F
        while self.stage_b and self.stage_b[0][0] <= b - 3:  # (no-ops in steady state)
            self._stage_b()
        while self.stage_c and self.stage_c[0][0] <= b - 3:
            self._stage_c()
        if self.direct and b - 3 in self.decoded_ev and self.cuda:
            ev = self.decoded_ev[b - 3]
            for st in streams:
                st.wait_event(ev)
        if self.fused and b - 3 in self.gathered_ev and self.cuda:  # the trace writes wire b % 3,
            ev = self.gathered_ev[b - 3]                           # last read by gather b-3
            for st in streams:
                st.wait_event(ev)

    # -- stages -------------------------------------------------------------------
    def _spec_bytes(self, n_frames):
        """Speculative gather size of a batch: capacity per frame x frames, at least the wire's fixed
        part (headers: a decode of a wire cut short then reads only stale payload, inside the slot)."""
        n = int(self.capacity_per_frame * n_frames)
        n = max(n, int(self.layout_fn(n_frames).fixed_bytes))
        return min(self.rank_stride, (n + 7) // 8 * 8)

    def _stage_a(self, main, n_frames):
        import torch.distributed as dist
        b = self.batch
        if self.solo:  # the frames are final as traced (stream order)
            self.batch += 1
            if self.root:
                self.decoded += 1
            return
        i = b % 3
        while self.stage_b and self.stage_b[0][0] <= b - 3:  # (no-ops in steady state)
            self._stage_b()
        while self.stage_c and self.stage_c[0][0] <= b - 3:
            self._stage_c()
        for pb, _, _, _ in self.pending_checks:
            if b - pb >= 3:  # this encode would overwrite size/wire slot i before pb's deferred check read it
                raise RuntimeError(f"batch {b}: batch {pb}'s deferred size check is still pending "
                                   f"(defer_checks allows runs of at most three batches; call check_deferred)")
        # an empty pipeline (a run's first batch; all of a short run): speculative gather first
        first = self.capacity_per_frame is not None and not self.stage_b and not self.stage_c
        if b - 3 in self.gathered_ev:  # wire i was last read by gather b-3
            ev = self.gathered_ev.pop(b - 3)
            if self.cuda:
                main.wait_event(ev)
        if self.direct or self.idle:
            self.size[i].zero_()  # nothing to ship: rank 0's bands are in its frames (or it has none)
        else:
            self.encode(None if self.fused else self.raw[b % 2], n_frames, self.wire[i], self.size[i], main)
        if self.cuda:  # (events reused round robin: a wait takes the state recorded before it)
            ev = self.enc_events[b % len(self.enc_events)]
            ev.record(main)
            self.encoded_ev[b] = ev
            for old in [x for x in self.encoded_ev if x < b - 3]:
                del self.encoded_ev[old]
        if first:
            # the gather right behind the encode and the size reduce after it, so that neither the
            # reduce nor its read-back sits between the encode and the decode: stage C decodes, then
            # checks the reduced size (and gathers + decodes again if it was exceeded).  A deferred
            # check (defer_checks, GPUs) reduces the size only after the caller's region has ended
            # (check_deferred): no collective between this batch's gather and its decode at all
            n = self._spec_bytes(n_frames)
            gw = self._gather(b, i, n)
            work = None if (self.defer_checks and self.cuda) else self._size_reduce(i)
            self.stage_c.append((b, n_frames, gw, (work, n, True)))
        else:
            work = self._size_reduce(i)
            self.stage_b.append((b, n_frames, work))
        self.batch += 1
    def _size_reduce(self, i):
        import torch.distributed as dist
        if self.coll is not None:
            return self.coll.all_reduce_max(self.size[i], self.comm)
        return dist.all_reduce(self.size[i], op=dist.ReduceOp.MAX, async_op=True)

    def _stage_b(self):
        b = self.stage_b[0][0]
        while self.stage_c and self.stage_c[0][0] <= b - 2:  # receive buffer b % 2 is free again
            self._stage_c()
        b, n_frames, work = self.stage_b.pop(0)
        i = b % 3
        # (the exact size even with set_capacity: in a pipeline the reduce of batch b-1 completed
        # while batch b was traced, and a speculative gather would move the margin over the links
        # too -- world-1 rehearsal at 1024 frames: 19.9-20.0 us/frame exact, 20.5-20.7 speculative)
        n = self._read_size(i, work)
        self.max_per_frame = max(self.max_per_frame, n / n_frames)
        self.bytes_sent += n
        self.stage_c.append((b, n_frames, self._gather(b, i, n), None))

    def _stage_c(self):
        b, n_frames, gw, spec = self.stage_c.pop(0)
        if spec is None:
            self._decode(b, n_frames, gw)
        else:  # speculative gather: the reduced size decides whether it sufficed
            work, n_spec, decode_first = spec
            if decode_first:  # (a wire cut short decodes stale payload bytes inside its own slot)
                self.provisional.add(b)
                self._decode(b, n_frames, gw)
            if decode_first and self.defer_checks and self.cuda:
                self.pending_checks.append((b, n_frames, n_spec, b % 3))  # size reduced in check_deferred
                self.bytes_sent += n_spec
                if self.root:
                    self.decoded += 1
                return
            n = self._read_size(b % 3, work)
            self.max_per_frame = max(self.max_per_frame, n / n_frames)
            self.bytes_sent += n_spec
            if n > n_spec:  # some wire outgrew it (every rank sees the same n): gather again, in full
                self.redone += 1  # (after a decode that read the buffer; collectives run in issue order)
                gw = self._gather(b, b % 3, n, reader=b if decode_first else None)
                self.bytes_sent += n
            if n > n_spec or not decode_first:
                self._decode(b, n_frames, gw)
            self.provisional.discard(b)  # the decode that stands has been issued
        if self.root:
            self.decoded += 1

    def check_deferred(self):
        """After the caller's device synchronisation, on every rank: the deferred size checks
        (defer_checks) -- each batch's size reduce is issued here, outside the caller's region.  Returns
        True when every speculative gather sufficed (the batches are final); False when some wire
        outgrew its gather (every rank sees the same reduced size, so every rank returns the same) --
        those batches move to `abandoned` (ring_of refuses them for good: their ring slots are reused by
        later batches) and the run must be repeated without speculation.  A deferred run spans at most
        three batches: _stage_a raises before a fourth batch would overwrite a pending check's size slot."""
        ok = True
        for b, n_frames, n_spec, i in self.pending_checks:
            # the wire sizes' maximum over ranks (collective: every rank checks alike), then read back
            n = self._read_size(i, self._size_reduce(i))
            self.max_per_frame = max(self.max_per_frame, n / n_frames)
            if n > n_spec:
                ok = False
                self.deferred_failed += 1  # (not a redone batch: the caller repeats the whole run)
                self.abandoned.add(b)       # never final; its ring slot is reused by later batches
            self.provisional.discard(b)
        self.pending_checks = []
        return ok

    def _decode(self, b, n_frames, gw):
        """Rank 0: after gather `gw`, decode batch b's wires into frame ring b % 3 (on `dec`).  A
        speculative batch that outgrew its gather is decoded twice; the second decode is the one
        that stands (`decode_batch` names the batch being decoded)."""
        import torch
        self.decode_batch = b
        self.decodes_of[b] = self.decodes_of.get(b, 0) + 1
        if self.cuda:
            with torch.cuda.stream(self.dec):
                gw.wait()
                ev = torch.cuda.Event()
                ev.record(self.dec)
                self.gathered_ev[b] = ev
                if self.root:
                    self.decode(self.recv[b % 2], self.rank_stride, n_frames, self.frames[b % 3], self.dec,
                                self.first_rank)
                    dv = torch.cuda.Event()
                    dv.record(self.dec)
                    self.decoded_ev[b] = dv
        else:
            gw.wait()
            self.gathered_ev[b] = None
            if self.root:
                self.decode(self.recv[b % 2], self.rank_stride, n_frames, self.frames[b % 3], None, self.first_rank)
                self.decoded_ev[b] = None

    def commit(self, main=None):
        """Frame k traced (on `main`'s stream or joined into it).  At a batch end: stages A, B, C."""
        self.k += 1
        if self.k % self.F == 0:
            self._stage_a(main, self.F)
            if len(self.stage_b) > 1:
                self._stage_b()
            if len(self.stage_c) > 1:
                self._stage_c()

    def drain(self, main=None):
        if self.k % self.F:
            self._stage_a(main, self.k % self.F)
            self.k += self.F - self.k % self.F
        while self.stage_b:
            self._stage_b()
        while self.stage_c:
            self._stage_c()


class _Done:
    """A collective issued on the stream that consumes it: nothing to wait for."""

    def wait(self):
        return None


class CommUnavailable(RuntimeError):
    """Every rank agreed that the library communicator cannot be built (raised on all ranks alike)."""


class LibraryCollectives:
    """TileBandGather's two exchange steps through the HIP library's own communicator (rt_comm_*:
    RCCL on the caller's stream) instead of torch.distributed's collective stream.

    Every rank builds one; construction is collective over the process group, whose
    `broadcast(tensor)` (from rank 0) and `agree_min(int) -> int` (minimum over ranks) it uses:
      1. every rank probes RCCL (rt_comm_probe: loads it, creates nothing) and the ranks agree on
         the minimum -- if any rank cannot load it, every rank raises CommUnavailable;
      2. rank 0 makes the unique id and ALWAYS broadcasts (flag byte + id; flag 0 when making the
         id failed), so every rank reaches the same broadcast -- a flag of 0 raises CommUnavailable
         on every rank;
      3. rt_comm_init on every rank (collective inside RCCL).
    Steps 1-2 make each decision from values every rank holds, so no rank enters rt_comm_init
    while another has given up (rank 0 raising before the broadcast hung the others).
    A failure inside rt_comm_init itself raises only on that rank; the caller agrees on the
    outcome afterwards (bench.py all_reduces an ok flag)."""

    def __init__(self, ctx, rank, world, broadcast, agree_min, device="cuda"):
        import torch
        if agree_min(1 if ctx.comm_probe() else 0) == 0:
            raise CommUnavailable("librccl cannot be loaded on some rank")
        msg = torch.zeros(1 + 128, dtype=torch.uint8, device=device)
        if rank == 0:
            try:
                uid = ctx.comm_unique_id()
                msg[1:].copy_(torch.frombuffer(bytearray(uid), dtype=torch.uint8))
                msg[0] = 1
            except Exception:  # noqa: BLE001 -- reported to every rank through the flag
                msg[0] = 0
        broadcast(msg)
        host = msg.cpu().numpy()
        if int(host[0]) != 1:
            raise CommUnavailable("rank 0 could not make an RCCL unique id")
        ctx.comm_init(world, rank, bytes(host[1:].tobytes()))
        self.ctx = ctx

    def all_reduce_max(self, t, stream):
        self.ctx.comm_allreduce_max_i64(t.data_ptr(), t.numel(), stream.cuda_stream)
        return _Done()

    def gather(self, send, n, recv, stride, rotate, stream):
        self.ctx.comm_gather(send.data_ptr(), n, recv.data_ptr() if recv is not None else 0, stride, rotate,
                             stream.cuda_stream)
        return _Done()
