"""Tile codec of the multi-GPU gather (raytracer_hip/tilecodec.py, the format spec and host
mirror of rt_encode_bands / rt_decode_gathered): lossless round trips over band layouts, ragged
sizes, several frames per wire and adversarial images; the C ABI's wire geometry
(rt_wire_layout_of, host only) matches the mirror.  GPU parity of the kernels against these
exact bytes is in test_gpu_codec.py."""
import os

import numpy as np
import pytest

from raytracer_hip import tilecodec as tc
from raytracer_hip.dist import RowBands

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def band_sets(frames, band_rows, world):
    """[F, H, W] frames -> per rank the [F * slot_elems] band sets (unused rows = garbage)."""
    F, H, W = frames.shape
    out = []
    for r in range(world):
        rb = RowBands(W, H, band_rows, r, world)
        s = np.full((F, rb.slot_elems // W, W), 0x3C3C3C, dtype=np.int32)
        for l0, y0, n in rb.row_spans():
            s[:, l0:l0 + n] = frames[:, y0:y0 + n]
        out.append(s.reshape(-1))
    return out


def roundtrip(frames, band_rows, world):
    F, H, W = frames.shape
    got = np.full((F, H, W), -1, dtype=np.int32)
    total = 0
    for r, bs in enumerate(band_sets(frames, band_rows, world)):
        wire = tc.encode(bs, W, H, band_rows, r, world, F)
        lay = tc.layout(W, H, band_rows, world, F)
        assert lay.fixed_bytes <= len(wire) <= lay.max_bytes and len(wire) % 8 == 0
        total += len(wire)
        tc.decode_into(got, wire, W, H, band_rows, r, world)
    assert np.array_equal(got, frames)
    return total


@pytest.mark.parametrize("name", ["frame_C2_96x54", "frame_C3_96x54", "frame_C4_64x36", "frame_REF_128"])
@pytest.mark.parametrize("band_rows,world", [(8, 1), (8, 2), (8, 3), (4, 5), (16, 2), (3, 4)])
def test_roundtrip_golden_frames(name, band_rows, world):
    img = np.load(os.path.join(GOLDEN, name + ".npy")).astype(np.int32)
    roundtrip(img[None], band_rows, world)


@pytest.mark.parametrize("W,H,band_rows,world", [(1, 1, 8, 1), (7, 5, 8, 2), (9, 17, 8, 3), (33, 65, 5, 8),
                                                 (64, 8, 8, 1), (15, 40, 8, 9), (100, 3, 1, 2)])
def test_roundtrip_ragged_and_random(W, H, band_rows, world):
    rng = np.random.default_rng(W * 1000 + H)
    noise = rng.integers(0, 1 << 24, size=(2, H, W)).astype(np.int32)
    smooth = (np.add.outer(np.arange(H), np.arange(W)) * 0x010203 & 0xFFFFFF).astype(np.int32)[None]
    roundtrip(np.concatenate([noise, smooth, np.zeros((1, H, W), np.int32)]), band_rows, world)


def test_flat_frame_has_no_payload_and_noise_fits_capacity():
    W, H = 64, 48
    lay = tc.layout(W, H, 8, 1, 1)
    flat = np.full((H * W,), 0x123456, dtype=np.int32)
    wire = tc.encode(flat, W, H, 8, 0, 1)
    assert len(wire) == lay.fixed_bytes and np.frombuffer(wire[:4], np.uint32)[0] == 0
    rng = np.random.default_rng(1)
    # extreme residuals (+-128 alternating) need all 8 bits: the payload is the capacity
    worst = np.where(np.add.outer(np.arange(H), np.arange(W)) % 2 == 0, 0, 0x808080).astype(np.int32)
    assert len(tc.encode(worst.reshape(-1), W, H, 8, 0, 1)) == lay.max_bytes
    assert len(tc.encode(rng.integers(0, 1 << 24, H * W).astype(np.int32), W, H, 8, 0, 1)) <= lay.max_bytes


def test_top_byte_is_ignored():
    W, H = 16, 16
    img = (np.arange(W * H, dtype=np.int64) * 0x010101 & 0xFFFFFF).astype(np.int32)
    dirty = (img.astype(np.int64) | (0x7F << 24)).astype(np.int32)
    assert tc.encode(img, W, H, 8, 0, 1) == tc.encode(dirty, W, H, 8, 0, 1)


def test_compression_on_rendered_frames():
    """The point of the codec: rendered frames are mostly flat (small frames less so; C2 at
    1920x1080 compresses 12.9x)."""
    for name, floor in (("frame_C2_96x54", 1.5), ("frame_REF_128", 1.5)):
        img = np.load(os.path.join(GOLDEN, name + ".npy")).astype(np.int32)
        H, W = img.shape
        total = roundtrip(img[None], 8, 2)
        assert 3 * H * W / total > floor, (name, 3 * H * W / total)


@pytest.mark.parametrize("W,H,band_rows,world,F", [(1920, 1080, 8, 1, 1), (1920, 1080, 8, 8, 8), (7680, 4320, 8, 2, 8),
                                                   (33, 65, 5, 8, 3), (1, 1, 8, 1, 1), (100, 3, 1, 2, 4)])
def test_c_abi_wire_layout_matches_mirror(rtlib, W, H, band_rows, world, F):
    from raytracer_hip import wire_layout
    got = wire_layout(W, H, band_rows, world, F)
    want = tc.layout(W, H, band_rows, world, F)
    assert (got.fixed_bytes, got.max_bytes, got.tiles_x, got.tiles_y, got.tiles_per_frame, got.n_frames,
            got.n_tiles, got.n_chunks) == (want.fixed_bytes, want.max_bytes, want.tiles_x, want.tiles_y,
                                           want.tiles_per_frame, want.n_frames, want.n_tiles, want.n_chunks)


def test_c_abi_wire_layout_rejects_bad_arguments(rtlib):
    from raytracer_hip import RayTracerError, wire_layout
    for args in ((0, 8, 8, 1, 1), (8, 8, 0, 1, 1), (8, 8, 8, 0, 1), (8, 8, 8, 1, 0)):
        with pytest.raises(RayTracerError):
            wire_layout(*args)
