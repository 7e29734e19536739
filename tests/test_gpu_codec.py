"""GPU parity of the tile codec kernels (rt_encode_bands / rt_decode_gathered, csrc/rt_codec.hip):
the device wire equals the host mirror's bytes (tilecodec.py) exactly -- the layout is
deterministic -- and decoding every rank's wire reproduces the frame bit for bit, from
synthetic images and from the trace kernel's own band sets."""
import os

import numpy as np
import pytest

from raytracer_hip import scenes
from raytracer_hip import tilecodec as tc
from raytracer_hip.dist import RowBands

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _frames(kind, F, H, W, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 1 << 24, size=(F, H, W)).astype(np.int32)
    if kind == "flat":
        return np.full((F, H, W), 0x2B2B2B, dtype=np.int32)
    if kind == "golden":
        img = np.load(os.path.join(GOLDEN, "frame_C3_96x54.npy")).astype(np.int32)
        img = np.tile(img, (-(-H // img.shape[0]), -(-W // img.shape[1])))[:H, :W]
        return np.stack([np.roll(img, 3 * f, axis=1) for f in range(F)])
    base = (np.add.outer(np.arange(H) * 3, np.arange(W)) & 255)
    return np.stack([((base + f) * 0x010101 + rng.integers(0, 3, size=(H, W))) & 0xFFFFFF
                     for f in range(F)]).astype(np.int32)


def _band_set(frames, band_rows, rank, world):
    F, H, W = frames.shape
    rb = RowBands(W, H, band_rows, rank, world)
    s = np.full((F, rb.slot_elems // W, W), 0x7E5A3C, dtype=np.int32)  # unused rows: garbage
    for l0, y0, n in rb.row_spans():
        s[:, l0:l0 + n] = frames[:, y0:y0 + n]
    return rb, s.reshape(-1)


@pytest.mark.parametrize("kind", ["golden", "smooth", "noise", "flat"])
@pytest.mark.parametrize("W,H,band_rows,world,F", [(96, 54, 8, 2, 1), (100, 37, 4, 3, 3), (1, 1, 8, 1, 1),
                                                   (33, 65, 5, 8, 2), (257, 130, 8, 1, 2), (64, 16, 8, 4, 5)])
def test_device_wire_equals_host_mirror_and_decodes(gpu_ctx, kind, W, H, band_rows, world, F):
    import torch
    frames = _frames(kind, F, H, W, seed=W + H + F)
    lay = tc.layout(W, H, band_rows, world, F)
    stride = (lay.max_bytes + 255) // 256 * 256
    gathered = torch.zeros(world * stride, dtype=torch.uint8, device="cuda")
    size = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for r in range(world):
        rb, bs = _band_set(frames, band_rows, r, world)
        d_bs = torch.from_numpy(bs).cuda()
        wire = gathered[r * stride:(r + 1) * stride]
        wire.fill_(0xCD)
        gpu_ctx.encode_bands(W, H, band_rows, r, world, d_bs.data_ptr(), rb.slot_elems, F, wire.data_ptr(),
                             size.data_ptr(), s)
        torch.cuda.synchronize()
        want = tc.encode(bs, W, H, band_rows, r, world, F)
        assert int(size.item()) == len(want)
        got = wire[:len(want)].cpu().numpy().tobytes()
        assert got == want, f"rank {r}: wire differs from the host mirror"
    out = torch.full((F * H * W,), -1, dtype=torch.int32, device="cuda")
    gpu_ctx.decode_gathered(W, H, band_rows, world, gathered.data_ptr(), stride, F, out.data_ptr(), H * W, s)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(F, H, W), frames)


@pytest.mark.parametrize("cfg,world,band_rows,rank0_direct", [("C2", 2, 8, True), ("C3", 8, 8, True), ("C4", 3, 8, False),
                                                              ("REF", 5, 4, True), ("C2", 1, 8, False)])
def test_traced_band_sets_roundtrip_to_the_frame(gpu_ctx, cfg, world, band_rows, rank0_direct):
    """The N>1 data path on one GPU: every simulated rank traces its band set (rt_render_bands),
    encodes it, rank 0 decodes all wires -> identical to the single-launch frame.  With
    rank0_direct, rank 0 renders its rows straight into the frame (RT_BANDS_FRAME) and the
    decode starts at rank 1 (bench.py's default)."""
    import torch
    from raytracer_hip import abi
    sc = scenes.config(cfg)
    if cfg != "C2":
        sc = sc.resized(640, 360)
    W, H = sc.width, sc.height
    gpu_ctx.set_scene(sc)
    full = gpu_ctx.render(W, H).copy()
    lay = tc.layout(W, H, band_rows, world, 1)
    stride = (lay.max_bytes + 255) // 256 * 256
    gathered = torch.zeros(world * stride, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    total = 0
    frame = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
    first = 1 if rank0_direct else 0
    if rank0_direct:
        gpu_ctx.render_bands_ex(W, H, band_rows, 0, world, frame.data_ptr(), abi.RT_BANDS_FRAME, s)
    for r in range(first, world):
        rb = RowBands(W, H, band_rows, r, world)
        buf = torch.zeros(rb.slot_elems, dtype=torch.int32, device="cuda")
        gpu_ctx.render_bands_ex(W, H, band_rows, r, world, buf.data_ptr(), abi.RT_BANDS_INT32, s)
        size = torch.zeros(1, dtype=torch.int64, device="cuda")
        gpu_ctx.encode_bands(W, H, band_rows, r, world, buf.data_ptr(), rb.slot_elems, 1,
                             gathered[r * stride:].data_ptr(), size.data_ptr(), s)
        torch.cuda.synchronize()
        total += int(size.item())
    gpu_ctx.decode_gathered(W, H, band_rows, world, gathered.data_ptr(), stride, 1, frame.data_ptr(), W * H, s,
                            first_rank=first)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().reshape(H, W), full)
    assert total < 3 * W * H  # smaller than the RGB24 band sets


@pytest.mark.parametrize("cfg,size,world,band_rows,F,splits", [
    ("C2", (1920, 1080), 2, 8, 2, (2,)), ("C3", (640, 360), 3, 8, 4, (1, 2)), ("C4", (320, 180), 4, 8, 2, (2,)),
    ("REF", (203, 97), 3, 5, 3, (3,)), ("C2", (131, 67), 1, 8, 4, (1, 1, 2)), ("C4", (96, 54), 8, 4, 2, (1, 1))])
def test_fused_encoder_wire_equals_host_mirror(gpu_ctx, cfg, size, world, band_rows, F, splits):
    """rt_render_bands_tiles (the encoder fused into the trace kernels' epilogue, the band set never
    written) + rt_finish_wire give every rank the same bytes as the host mirror's encoding of the
    rank's traced band set -- direct and bundle kernels, ragged frames, band heights other than 8,
    ranks with fewer bands (their untraced tile rows), a batch traced in several launches and a
    finish over fewer frames than the batch holds.  The scratch and wire start dirty."""
    import torch
    from raytracer_hip import abi
    sc = scenes.config(cfg).resized(*size)
    W, H = size
    gpu_ctx.set_scene(sc)
    s = torch.cuda.current_stream().cuda_stream
    lay = tc.layout(W, H, band_rows, world, F)
    n = sum(splits)  # frames traced (<= F)
    for r in range(world):
        rb = RowBands(W, H, band_rows, r, world)
        buf = torch.zeros(rb.slot_elems, dtype=torch.int32, device="cuda")
        gpu_ctx.render_bands_ex(W, H, band_rows, r, world, buf.data_ptr(), abi.RT_BANDS_INT32, s)
        torch.cuda.synchronize()
        bs = np.tile(buf.cpu().numpy(), n)  # every frame of the batch has the same camera
        want = tc.encode(bs, W, H, band_rows, r, world, n)
        wire = torch.full((lay.max_bytes + 8,), 0xA5, dtype=torch.uint8, device="cuda")
        size_t = torch.zeros(1, dtype=torch.int64, device="cuda")
        f0 = 0
        for m in splits:
            gpu_ctx.render_bands_tiles(W, H, band_rows, r, world, f0, m, F, wire.data_ptr(), s)
            f0 += m
        gpu_ctx.finish_wire(W, H, band_rows, r, world, n, wire.data_ptr(), size_t.data_ptr(), s)
        torch.cuda.synchronize()
        assert int(size_t.item()) == len(want), (r, int(size_t.item()), len(want))
        assert wire[:len(want)].cpu().numpy().tobytes() == want, f"rank {r}: fused wire differs from the host mirror"


def test_fused_encoder_rejects_bad_arguments(gpu_ctx):
    import torch
    from raytracer_hip import RayTracerError
    wire = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    with pytest.raises(RayTracerError):  # frames past the batch
        gpu_ctx.render_bands_tiles(64, 64, 8, 0, 1, 1, 2, 2, wire.data_ptr())
    with pytest.raises(RayTracerError):  # rank out of range
        gpu_ctx.render_bands_tiles(64, 64, 8, 2, 2, 0, 1, 1, wire.data_ptr())
    with pytest.raises(RayTracerError):  # misaligned wire
        gpu_ctx.render_bands_tiles(64, 64, 8, 0, 1, 0, 1, 1, wire.data_ptr() + 4)


def test_finish_wire_only_finishes_the_staged_batch(gpu_ctx):
    """rt_finish_wire compacts the codec scratch of the batch rt_render_bands_tiles staged
    last -- another geometry, rank, wire, more frames than the batch, or a batch whose scratch an
    rt_encode_bands has reused since, is an error instead of a wire made of stale scratch."""
    import torch
    from raytracer_hip import RayTracerError
    gpu_ctx.set_scene(scenes.config("C2").resized(96, 64))
    wire = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    other = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    size_t = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu_ctx.render_bands_tiles(96, 64, 8, 1, 2, 0, 2, 3, wire.data_ptr())
    for args in [(96, 64, 8, 0, 2, 2, wire), (96, 64, 8, 1, 3, 2, wire), (96, 48, 8, 1, 2, 2, wire),
                 (96, 64, 4, 1, 2, 2, wire), (96, 64, 8, 1, 2, 2, other), (96, 64, 8, 1, 2, 4, wire)]:
        with pytest.raises(RayTracerError):
            gpu_ctx.finish_wire(*args[:6], args[6].data_ptr(), size_t.data_ptr())
    gpu_ctx.finish_wire(96, 64, 8, 1, 2, 2, wire.data_ptr(), size_t.data_ptr())  # the staged batch itself
    torch.cuda.synchronize()
    assert int(size_t.item()) > 0
    bands = torch.zeros(96 * 64, dtype=torch.int32, device="cuda")
    gpu_ctx.encode_bands(96, 64, 8, 1, 2, bands.data_ptr(), 96 * 32, 1, other.data_ptr(), size_t.data_ptr())
    with pytest.raises(RayTracerError):  # the scratch now holds that encode's segments
        gpu_ctx.finish_wire(96, 64, 8, 1, 2, 2, wire.data_ptr(), size_t.data_ptr())
    torch.cuda.synchronize()


def test_encode_rejects_bad_arguments(gpu_ctx):
    import torch
    from raytracer_hip import RayTracerError
    buf = torch.zeros(64 * 64, dtype=torch.int32, device="cuda")
    wire = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(RayTracerError):  # rank out of range
        gpu_ctx.encode_bands(64, 64, 8, 2, 2, buf.data_ptr(), 64 * 32, 1, wire.data_ptr())
    with pytest.raises(RayTracerError):  # frame stride smaller than the band set
        gpu_ctx.encode_bands(64, 64, 8, 0, 1, buf.data_ptr(), 64, 1, wire.data_ptr())
    with pytest.raises(RayTracerError):  # misaligned wire
        gpu_ctx.encode_bands(64, 64, 8, 0, 1, buf.data_ptr(), 64 * 64, 1, wire.data_ptr() + 4)


@pytest.mark.parametrize("fmt_name,world,rank", [("RT_BANDS_FRAME", 1, 0), ("RT_BANDS_FRAME", 3, 0), ("RT_BANDS_INT32", 2, 1),
                                                 ("RT_BANDS_RGB24", 3, 2)])
def test_batched_band_launch_equals_single_frames(gpu_ctx, fmt_name, world, rank):
    """rt_render_bands_batch: n frames in one launch (grid z), each bit-identical to the
    single-frame launch and written at its own stride; ray counters scale with n."""
    import torch
    from raytracer_hip import abi
    fmt = getattr(abi, fmt_name)
    sc = scenes.config("C3").resized(200, 120)
    W, H, br, n = sc.width, sc.height, 8, 3
    gpu_ctx.set_scene(sc)
    rb = RowBands(W, H, br, rank, world)
    per = W * H * 4 if fmt == abi.RT_BANDS_FRAME else rb.slot_elems * (3 if fmt == abi.RT_BANDS_RGB24 else 4)
    stride = (per + 255) // 256 * 256 + 256
    one = torch.full((stride,), 0x5A, dtype=torch.uint8, device="cuda")
    many = torch.full((n * stride,), 0x5A, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    gpu_ctx.reset_stats()
    gpu_ctx.render_bands_ex(W, H, br, rank, world, one.data_ptr(), fmt, s)
    torch.cuda.synchronize()
    st1 = gpu_ctx.stats()
    gpu_ctx.reset_stats()
    gpu_ctx.render_bands_batch(W, H, br, rank, world, n, many.data_ptr(), stride, fmt, s)
    torch.cuda.synchronize()
    stn = gpu_ctx.stats()
    want = one.cpu().numpy()
    got = many.cpu().numpy().reshape(n, stride)
    for f in range(n):
        assert np.array_equal(got[f], want), f"frame {f} differs"
    for k in ("primary_rays", "reflect_rays", "shadow_rays"):
        assert stn[k] == n * st1[k], k
