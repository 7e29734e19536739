"""GPU tests of the plugin surface's multi-GPU Tick (ABI 9), every call through the C ABI.

The reference's Tick() fills Surface.pixels and returns with the frame complete (RayTracer.cs:886-901,
template.cs:179,188-193).  With n band workers every worker traces its interleaved 8-row bands (band b
on worker b % n) and copies them into the caller's frame over its own device's PCIe link -- no gather
to one device, no single-link copy of the whole frame.  On a one-GPU box the n workers run as streams of
one device (RT_CREATE_SHARED_DEVICE): the band geometry, the per-worker copy jobs into one registered
buffer, the chunked synchronous hand-off and the double-buffered async path are the same code the
n-device context runs.  Bars: every frame's CRC = tests/golden/golden.json (full-size C2-C5), or every
pixel = the oracle's (ragged sizes, camera sweeps).  The RCCL gather path (RT_CREATE_RCCL_GATHER) is
forced on one GPU for C2/C3/C5.
"""
import os
import zlib

import numpy as np
import pytest

from raytracer_hip import Context, abi, scenes

pytestmark = pytest.mark.gpu


def crc(a):
    return f"{zlib.crc32(np.ascontiguousarray(a, dtype=np.int32).tobytes()) & 0xFFFFFFFF:08x}"


GUARD = 4096  # int32 sentinels on both sides of every host frame: a hand-off must not write outside it
SENTINEL = 0x5A5A5A5A


def guarded(n):
    """(buffer, frame): frame = the middle n int32 of buffer (16-byte aligned), the rest sentinels."""
    buf = np.full(n + 2 * GUARD, SENTINEL, dtype=np.int32)
    px = buf[GUARD:GUARD + n]
    px[:] = -1
    return buf, px


def check_guard(buf):
    assert (buf[:GUARD] == SENTINEL).all() and (buf[-GUARD:] == SENTINEL).all(), "write outside the host frame"


def _stats(ctx):
    st = ctx.stats()
    return {k: st[k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}


def _env_fixture(name):
    old = os.environ.get(name)

    def set_(v):
        if v is None:
            os.environ.pop(name, None)
        else:
            os.environ[name] = str(v)
    yield set_
    set_(old)


@pytest.fixture
def chunks_env():
    """Set RT_TICK_CHUNKS for one test (read by every rt_render), restored afterwards."""
    yield from _env_fixture("RT_TICK_CHUNKS")


@pytest.fixture
def copy_env():
    """Set RT_TICK_COPY (the synchronous hand-off: runtime / kernel / stream) for one test."""
    yield from _env_fixture("RT_TICK_COPY")


@pytest.fixture
def async_env():
    """Set RT_TICK_ASYNC (rt_render_async's hand-off: copy slice / copy engine on a second stream)."""
    yield from _env_fixture("RT_TICK_ASYNC")


@pytest.mark.parametrize("cid", ["C2", "C3", "C5"])
def test_rccl_gather_forced_path_golden(golden, cid):
    """rt_create_ex(1, RT_CREATE_RCCL_GATHER): rt_render traces 8-row bands, gathers them with ncclGather
    (a one-rank communicator from ncclCommInitAll), reassembles on device 0 and copies the frame --
    twice through one communicator; its counts are the golden's."""
    e = golden["cases"][cid]
    sc = scenes.config(cid)
    with Context(1, abi.RT_CREATE_RCCL_GATHER) as ctx:
        ctx.set_scene(sc)
        ctx.reset_stats()
        px = ctx.render(sc.width, sc.height).copy()
        assert crc(px) == e["crc32"]
        assert _stats(ctx) == {k: e["stats"][k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}
        assert crc(ctx.render(sc.width, sc.height)) == e["crc32"]
        ctx.set_timing(1)
        ctx.reset_stats()
        ctx.render(sc.width, sc.height)
        assert ctx.stats()["timed_gathers"] == 1


@pytest.mark.parametrize("cid", ["C2", "C3"])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 6, 7, 8])
def test_tick_workers_golden(golden, cid, world):
    """Simulated worlds 1..8: every worker's band set into ONE registered Surface.pixels buffer = the
    golden frame, with the golden's ray counts (summed over the workers)."""
    e = golden["cases"][cid]
    sc = scenes.config(cid)
    with Context(world, abi.RT_CREATE_SHARED_DEVICE) as ctx:
        ctx.set_scene(sc)
        buf, px = guarded(sc.width * sc.height)
        ctx.register_host(px)
        try:
            ctx.reset_stats()
            ctx.render(sc.width, sc.height, px)
            assert crc(px) == e["crc32"], f"{cid} world {world}"
            assert _stats(ctx) == {k: e["stats"][k] for k in ("primary_rays", "reflect_rays", "shadow_rays")}
            px[:] = -1  # a second Tick into the same buffer (buffers reused)
            ctx.render(sc.width, sc.height, px)
            assert crc(px) == e["crc32"]
            check_guard(buf)
        finally:
            ctx.unregister_host(px)


@pytest.mark.parametrize("mode", [None, "kernel", "runtime"])
@pytest.mark.parametrize("cid,world,chunks", [("C4", 1, None), ("C4", 2, 3), ("C4", 8, None), ("C5", 1, None),
                                              ("C5", 1, 3), ("C5", 2, None), ("C5", 8, 2), ("C2", 1, 4),
                                              ("C3", 3, 5)])
def test_tick_chunked_golden(golden, chunks_env, copy_env, cid, world, chunks, mode):
    """The synchronous Tick's chunked hand-off -- default: chunk c traced, then copied by the copy engine on
    a second stream while chunk c+1 is traced; kernel: chunk c's copy rides in chunk c+1's launch, the last
    by the copy kernel; runtime: one copy after the trace -- with the default chunk count (by share size:
    C5 at n = 1 takes 8) and forced counts, including more chunks than a worker has bands."""
    chunks_env(chunks)
    copy_env(mode)
    e = golden["cases"][cid]
    sc = scenes.config(cid)
    with Context(world, abi.RT_CREATE_SHARED_DEVICE) as ctx:
        ctx.set_scene(sc)
        buf, px = guarded(sc.width * sc.height)
        ctx.register_host(px)
        try:
            ctx.render(sc.width, sc.height, px)
            assert crc(px) == e["crc32"], f"{cid} world {world} chunks {chunks}"
            check_guard(buf)
        finally:
            ctx.unregister_host(px)


@pytest.mark.parametrize("world", [1, 3, 8])
def test_tick_unregistered_buffer(golden, world):
    """An unregistered host buffer: each worker's bands by the runtime's copies, one per band, and nothing
    written outside the frame (a pitched 2-D copy into pageable memory is not used: nothing bounds what its
    staging writes past the last row; it was not the cause of r05b's exit abort, profiles/r06_exit_abort.txt)."""
    e = golden["cases"]["C3"]
    sc = scenes.config("C3")
    with Context(world, abi.RT_CREATE_SHARED_DEVICE) as ctx:
        ctx.set_scene(sc)
        buf, px = guarded(sc.width * sc.height)
        ctx.render(sc.width, sc.height, px)
        assert crc(px) == e["crc32"]
        check_guard(buf)


@pytest.mark.parametrize("size", [(643, 357), (100, 9), (37, 1), (1, 61), (250, 131)])
@pytest.mark.parametrize("world", [1, 2, 3, 7])
@pytest.mark.parametrize("registered", [True, False])
def test_tick_ragged_vs_oracle(oracle, chunks_env, size, world, registered):
    """Ragged frames (height not a multiple of 8, so the frame's last band is cut; widths not a multiple of
    4, so a band set's length is not whole 16-byte stores; more workers than bands): every pixel = the
    oracle's.  Chunked too (RT_TICK_CHUNKS=2)."""
    W, H = size
    sc = scenes.config("C3").resized(W, H)
    want, _ = oracle.render(sc, oracle.MODE_NEAREST)
    with Context(world, abi.RT_CREATE_SHARED_DEVICE) as ctx:
        ctx.set_scene(sc)
        for chunks in (None, 2):
            chunks_env(chunks)
            buf, px = guarded(W * H)
            if registered:
                ctx.register_host(px)
            try:
                ctx.render(W, H, px)
            finally:
                if registered:
                    ctx.unregister_host(px)
            got = px.reshape(H, W)
            assert np.array_equal(got, want), f"{W}x{H} world {world} chunks {chunks}: {int((got != want).sum())} px"
            check_guard(buf)


@pytest.mark.parametrize("mode", [None, "slice", "stream"])
@pytest.mark.parametrize("world", [1, 2, 4, 7])
def test_tick_async_workers_vs_oracle(oracle, async_env, world, mode):
    """rt_render_async at n workers: 7 frames queued, a new camera each and the frame size changing twice
    mid-queue, each into its own registered buffer, ONE rt_wait -- every frame = the oracle's.  Every
    worker double-buffers its band set on its own stream; frame k's copy rides in frame k+1's launch (slice)
    or runs on the copy engine behind frame k's trace (stream; the default for large shares)."""
    async_env(mode)
    base = scenes.config("C3")
    sizes = [(320, 180)] * 3 + [(200, 113)] * 2 + [(320, 180)] * 2
    rng = np.random.default_rng(7)
    with Context(world, abi.RT_CREATE_SHARED_DEVICE) as ctx:
        ctx.set_scene(base.resized(*sizes[0]))
        bufs, wants, guards = [], [], []
        for k, (W, H) in enumerate(sizes):
            sc = base.resized(W, H)
            pos, yaw, pitch = base.camera
            cam = ((pos[0] + float(rng.uniform(-1, 1)), pos[1] + float(rng.uniform(0, 0.5)), pos[2]),
                   float(rng.uniform(-0.2, 0.2)), float(rng.uniform(-0.1, 0.1)))
            sc.camera = cam
            wants.append(oracle.render(sc, oracle.MODE_NEAREST)[0])
            ctx.set_camera(sc.c_camera())
            gb, px = guarded(W * H)
            ctx.register_host(px)
            bufs.append(px)
            guards.append(gb)
            ctx.render_async(W, H, px)
        ctx.wait()
        for k, (px, want) in enumerate(zip(bufs, wants)):
            W, H = sizes[k]
            got = px.reshape(H, W)
            assert np.array_equal(got, want), f"frame {k} world {world}: {int((got != want).sum())} px differ"
        # a frame still pending is flushed by a synchronous rt_render into the same buffer
        ctx.render_async(*sizes[0], bufs[0])
        ctx.render(*sizes[0], bufs[0])
        for px in bufs:
            ctx.unregister_host(px)
        assert np.array_equal(bufs[0].reshape(sizes[0][1], sizes[0][0]), wants[-1])
        for gb in guards:
            check_guard(gb)


@pytest.mark.parametrize("mode", [None, "slice", "stream"])
@pytest.mark.parametrize("cid", ["C3", "C5"])
def test_tick_async_workers_golden(golden, async_env, cid, mode):
    """Full-size double-buffered Ticks at 4 workers, two frames deep with a wait per pair (the display
    loop of bench.py's tick_async_*): both buffers = the golden frame after each wait."""
    async_env(mode)
    e = golden["cases"][cid]
    sc = scenes.config(cid)
    with Context(4, abi.RT_CREATE_SHARED_DEVICE) as ctx:
        ctx.set_scene(sc)
        gbs = [guarded(sc.width * sc.height) for _ in range(2)]
        bufs = [px for _, px in gbs]
        for b in bufs:
            ctx.register_host(b)
        try:
            for k in range(4):
                ctx.render_async(sc.width, sc.height, bufs[k % 2])
                if k % 2:
                    ctx.wait()
                    assert crc(bufs[0]) == e["crc32"] and crc(bufs[1]) == e["crc32"], f"pair {k // 2}"
                    for gb, _ in gbs:
                        check_guard(gb)
                    bufs[0][:] = -1
                    bufs[1][:] = -1
        finally:
            for b in bufs:
                ctx.unregister_host(b)


@pytest.mark.parametrize("world", [2, 5])
def test_render_device_workers_golden(golden, world):
    """rt_render_device with n workers on one device: each writes its bands straight into the device
    frame on its own stream, ordered after the caller's stream, which waits for all of them."""
    import torch
    e = golden["cases"]["C3"]
    sc = scenes.config("C3")
    with Context(world, abi.RT_CREATE_SHARED_DEVICE) as ctx:
        ctx.set_scene(sc)
        st = torch.cuda.current_stream()
        out = torch.full((sc.width * sc.height,), -1, dtype=torch.int32, device="cuda")
        ctx.render_device(sc.width, sc.height, out.data_ptr(), st.cuda_stream)
        got = out.cpu().numpy()  # (ordered on the caller's stream)
        assert crc(got) == e["crc32"]


def test_shared_device_refuses_rccl_gather():
    """RCCL refuses two ranks on one device: the flag combination is an argument error at creation."""
    from raytracer_hip import RayTracerError
    with pytest.raises(RayTracerError) as ei:
        Context(2, abi.RT_CREATE_SHARED_DEVICE | abi.RT_CREATE_RCCL_GATHER)
    assert ei.value.code == abi.RT_ERR_INVALID_ARG


CHILD_RCCL_THEN_TORCH = r"""
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "uu-infogr-raytracer_amd"))
from raytracer_hip import Context, abi, scenes
sc = scenes.config("C2").resized(320, 180)
with Context(1, abi.RT_CREATE_RCCL_GATHER) as c:  # loads librccl (our dlopen) before torch does
    c.set_scene(sc)
    c.render(sc.width, sc.height)
import torch  # torch's own librccl
torch.zeros(1, device="cuda").add_(1).sum().item()
print("child done", flush=True)
"""


def test_rccl_then_torch_in_a_fresh_process_exits_cleanly():
    """Round 5's exit abort in the order that produced it (profiles/r06_exit_abort.txt): a fresh interpreter loads
    RCCL through an RCCL-gather context and renders, then imports torch and runs one GPU op, then exits -- status
    0 and no glibc heap message.  (The parent pytest process may have imported torch already, which hides the
    order; the child starts clean and the parent makes no GPU call for it.)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", CHILD_RCCL_THEN_TORCH, root], capture_output=True, text=True, timeout=110)
    err = r.stderr.lower()
    assert r.returncode == 0, f"rc {r.returncode}: {r.stderr[-2000:]}"
    assert "child done" in r.stdout
    assert "double free" not in err and "corruption" not in err, r.stderr[-2000:]
